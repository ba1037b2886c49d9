// Throughput of one returning global atomicAdd per wave at kernel end, as a deal
// counter would use it: 4096 single-wave blocks, lane 0 adds 1 to one of M
// counters (block % M, each counter on its own 256-B line or packed in one line)
// and stores the returned slot.  Prints the kernel time per variant (HIP events).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_atomic(int* ctr, int* out, int m, int stride, int spin) {
    // a little independent work first so the atomics of the blocks do not all start at once
    float acc = threadIdx.x;
    for (int i = 0; i < spin; ++i) acc = acc * 1.0001f + 0.5f;
    if (threadIdx.x == 0) {
        int slot = m > 0 ? atomicAdd(&ctr[(blockIdx.x % m) * stride], 1) : (int)blockIdx.x;
        out[blockIdx.x] = slot + (acc == 1234.5f);
    }
}

int main() {
    const int B = 4096;
    int *ctr, *out;
    hipMalloc(&ctr, 1 << 20);
    hipMalloc(&out, B * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int ms[] = {0, 1, 8, 8, 32, 64};
    const int strides[] = {1, 1, 1, 64, 64, 64};
    for (int spin : {0, 2000}) {
        for (int v = 0; v < 6; ++v) {
            float best = 1e9f;
            for (int rep = 0; rep < 20; ++rep) {
                hipMemset(ctr, 0, 1 << 20);
                hipEventRecord(a);
                hipLaunchKernelGGL(k_atomic, dim3(B), dim3(64), 0, 0, ctr, out, ms[v], strides[v], spin);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float t;
                hipEventElapsedTime(&t, a, b);
                if (t < best) best = t;
            }
            std::vector<int> h(B);
            hipMemcpy(h.data(), out, B * 4, hipMemcpyDeviceToHost);
            long s = 0;
            for (int x : h) s += x;
            printf("spin %4d counters %2d stride %2d: %8.2f us (checksum %ld)\n", spin, ms[v], strides[v], best * 1e3, s);
        }
    }
    return 0;
}
