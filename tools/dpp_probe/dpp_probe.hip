// Diagnostic: DPP row-shift / row-broadcast inclusive scans over a wave64 on
// gfx950, checked against a host scan.  hipcc --offload-arch=gfx950 dpp_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <class Op>
__device__ inline int scan_dpp(int v, Op op) {
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true));
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true));
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true));
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true));
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));
    return v;
}

__global__ void k(const int* in, int* add, int* mx, int* stage) {
    const int l = threadIdx.x;
    const int v = in[l];
    add[l] = scan_dpp(v, [](int a, int b) { return a + b; });
    mx[l] = scan_dpp(v, [](int a, int b) { return a > b ? a : b; });
    // the individual steps
    int s = v;
    s = s + __builtin_amdgcn_update_dpp(0, s, 0x111, 0xf, 0xf, true); stage[0 * 64 + l] = s;
    s = s + __builtin_amdgcn_update_dpp(0, s, 0x112, 0xf, 0xf, true); stage[1 * 64 + l] = s;
    s = s + __builtin_amdgcn_update_dpp(0, s, 0x114, 0xf, 0xf, true); stage[2 * 64 + l] = s;
    s = s + __builtin_amdgcn_update_dpp(0, s, 0x118, 0xf, 0xf, true); stage[3 * 64 + l] = s;
    s = s + __builtin_amdgcn_update_dpp(0, s, 0x142, 0xa, 0xf, false); stage[4 * 64 + l] = s;
    s = s + __builtin_amdgcn_update_dpp(0, s, 0x143, 0xc, 0xf, false); stage[5 * 64 + l] = s;
}

int main() {
    int h[64], ha[64], hm[64], hs[6 * 64];
    srand(1);
    for (int i = 0; i < 64; ++i) h[i] = rand() % 7;
    int *d, *da, *dm, *ds;
    hipMalloc(&d, 256); hipMalloc(&da, 256); hipMalloc(&dm, 256); hipMalloc(&ds, 6 * 256);
    hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, da, dm, ds);
    hipMemcpy(ha, da, 256, hipMemcpyDeviceToHost);
    hipMemcpy(hm, dm, 256, hipMemcpyDeviceToHost);
    hipMemcpy(hs, ds, 6 * 256, hipMemcpyDeviceToHost);
    int bad = 0, acc = 0, m = 0;
    for (int i = 0; i < 64; ++i) {
        acc += h[i];
        m = h[i] > m ? h[i] : m;
        if (ha[i] != acc || hm[i] != m) { if (bad < 8) printf("lane %d: add %d want %d, max %d want %d\n", i, ha[i], acc, hm[i], m); ++bad; }
    }
    if (bad) for (int st = 0; st < 6; ++st) { printf("stage %d:", st); for (int i = 0; i < 64; ++i) printf(" %d", hs[st * 64 + i]); printf("\n"); }
    printf("input:"); for (int i = 0; i < 64; ++i) printf(" %d", h[i]); printf("\n");
    printf("%s (%d bad lanes)\n", bad ? "DPP SCAN MISMATCH" : "DPP SCAN OK", bad);
    return bad != 0;
}
