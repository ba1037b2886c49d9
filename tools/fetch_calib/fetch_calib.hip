// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths k_step uses (MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for
// 16-B-per-lane streaming reads, which it reports at exactly half).  Each kernel
// reads a known number of distinct bytes from a buffer larger than the 256 MB
// Infinity Cache; run under `rocprofv3 --pmc FETCH_SIZE` (and WRITE_SIZE), then
// compare the counter with the byte count printed here (tools/fetch_calib.py).
//   k_read16: 16 B per lane, fully coalesced (the guide's calibrated case)
//   k_read4 : 4 B per lane, fully coalesced
//   k_soa   : k_step's state pattern -- per wave, 8 lanes x 4 B from each of 16
//             SoA fields (32 B per field per wave), waves in plain block order
//   k_soa_x : the same with the XCD-aware block -> env order of k_step
//   k_write4: 4 B per lane coalesced stores (WRITE_SIZE)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_read16(const float4* __restrict__ src, size_t n4, float* out) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = src[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) out[0] = acc;  // keeps the loads, never true for the zeroed buffer
}
__global__ void k_read4(const float* __restrict__ src, size_t n, float* out) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += src[i];
    if (acc == 12345.f) out[0] = acc;
}
__device__ inline int xcd_env(int b, int E) {
    const int q = E >> 3;
    return b < 8 * q ? (b & 7) * q + (b >> 3) : b;
}
template <bool XCD>
__global__ void k_soa(const float* __restrict__ base, size_t stride, int E, int N, float* out) {
    const int e = XCD ? xcd_env((int)blockIdx.x, E) : (int)blockIdx.x;
    const int lane = threadIdx.x;
    float acc = 0.f;
    if (lane < N)
        for (int f = 0; f < 16; ++f) acc += base[(size_t)f * stride + (size_t)e * N + lane];
    if (acc == 12345.f) out[0] = acc;
}
__global__ void k_write4(float* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = 1.0f;
}

int main() {
    const size_t bytes = size_t(768) << 20;  // > 256 MB MALL
    char* buf;
    float* out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 0, bytes));
    CK(hipDeviceSynchronize());
    const size_t chunk = size_t(64) << 20;  // each kernel reads a fresh 64 MB region
    // 1. 16 B / lane, 64 MB
    hipLaunchKernelGGL(k_read16, dim3(4096), dim3(256), 0, 0, (const float4*)(buf), chunk / 16, out);
    // 2. 4 B / lane, 64 MB
    hipLaunchKernelGGL(k_read4, dim3(4096), dim3(256), 0, 0, (const float*)(buf + chunk), chunk / 4, out);
    // 3./4. k_step's SoA pattern: E = 4096 envs x N = 8 agents x 16 fields of 4 B = 2 MB each
    const int E = 4096, N = 8;
    const size_t stride = size_t(E) * N;  // elements between fields
    hipLaunchKernelGGL(k_soa<false>, dim3(E), dim3(64), 0, 0, (const float*)(buf + 2 * chunk), stride, E, N, out);
    hipLaunchKernelGGL(k_soa<true>, dim3(E), dim3(64), 0, 0, (const float*)(buf + 3 * chunk), stride, E, N, out);
    // 5. 4 B / lane stores, 64 MB
    hipLaunchKernelGGL(k_write4, dim3(4096), dim3(256), 0, 0, (float*)(buf + 4 * chunk), chunk / 4);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    printf("bytes: k_read16 %zu  k_read4 %zu  k_soa %zu  k_soa_x %zu  k_write4 %zu\n", chunk, chunk,
           size_t(16) * stride * 4, size_t(16) * stride * 4, chunk);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
