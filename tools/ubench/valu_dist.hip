// Microbenchmark: the KNNScanReduce A1 inner body (8 leaves x D dims of
// sequential sub/mul/add per lane, q broadcast from LDS) -- cycles per query
// per wave at 8 waves per CU (one block per CU via LDS size).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int D, int WAVES, bool LDSQ>
__global__ __launch_bounds__(64 * WAVES) void k(const float* __restrict__ in, float* __restrict__ out, int iters,
                                               unsigned long long* cyc) {
    extern __shared__ float sq[];
    const int tid = threadIdx.x;
    for (int i = tid; i < 1024 * D; i += blockDim.x) sq[i] = in[i % 4096];
    __syncthreads();
    float c[8][D];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int d = 0; d < D; ++d) c[s][d] = in[((tid * 8 + s) & 255) * D + d];
    uint32_t acc = 0;
    float qr[D];
#pragma unroll
    for (int d = 0; d < D; ++d) qr[d] = in[d];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
        float q[D];
        const float* qv = sq + (it & 1023) * D;
#pragma unroll
        for (int d = 0; d < D; ++d) q[d] = LDSQ ? qv[d] : qr[d] + (float)it;
        float dv[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) dv[s] = 0.0f;
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const float t = __fsub_rn(q[d], c[s][d]);
                dv[s] = __fadd_rn(dv[s], __fmul_rn(t, t));
            }
        uint32_t m = 0xffffffffu;
#pragma unroll
        for (int s = 0; s < 8; ++s) m = min(m, __float_as_uint(dv[s]));
        acc ^= m;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + tid] = __uint_as_float(acc);
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int D, int WAVES, bool LDSQ>
void run(const char* name, float* din, float* dout, unsigned long long* dc, int blocks) {
    const int iters = 20000;
    const size_t shm = 140 * 1024;
    hipFuncSetAttribute((const void*)k<D, WAVES, LDSQ>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipLaunchKernelGGL((k<D, WAVES, LDSQ>), dim3(blocks), dim3(64 * WAVES), shm, 0, din, dout, iters, dc);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL((k<D, WAVES, LDSQ>), dim3(blocks), dim3(64 * WAVES), shm, 0, din, dout, iters, dc);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    unsigned long long c0;
    hipMemcpy(&c0, dc, 8, hipMemcpyDeviceToHost);
    const double ops = 3.0 * D * 8 * 64 * WAVES * (double)iters;
    printf("%-28s blocks %3d: %.1f cyc/query/block  %.2f ms  %.3f Tops/s per CU-block, clock %.2f GHz\n", name, blocks,
           (double)c0 / iters, ms, ops / (ms * 1e-3) / 1e12, (double)c0 / (ms * 1e-3) / 1e9);
}

int main() {
    float *din, *dout;
    unsigned long long* dc;
    hipMalloc(&din, 4096 * 4);
    hipMalloc(&dout, 1 << 22);
    hipMalloc(&dc, 8 * 1024);
    float h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = (float)((i * 37) % 101) * 0.01f;
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    run<16, 8, true>("D16 8w ldsq", din, dout, dc, 1);
    run<16, 8, false>("D16 8w regq", din, dout, dc, 1);
    run<16, 4, true>("D16 4w ldsq", din, dout, dc, 1);
    run<16, 8, true>("D16 8w ldsq", din, dout, dc, 256);
    run<8, 8, true>("D8 8w ldsq", din, dout, dc, 1);
    return 0;
}
