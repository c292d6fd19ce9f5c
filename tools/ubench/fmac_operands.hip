// Issue rate of v_fmac_f32 with the multiplier in a VGPR (three VGPR reads)
// vs in an SGPR (two VGPR reads), 8 waves per CU as in the scan kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <bool SGPR>
__global__ __launch_bounds__(512) void k(const float* in, float* out, long long* cyc, int iters) {
    float c[16], acc[16];
    for (int s = 0; s < 16; ++s) {
        c[s] = in[(threadIdx.x + s) & 511];
        acc[s] = 0.0f;
    }
    float qv = in[threadIdx.x & 3];
    __syncthreads();
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            if constexpr (SGPR) {
                const float qs = __builtin_amdgcn_readfirstlane(qv);
#pragma unroll
                for (int s = 0; s < 16; ++s) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(acc[s]) : "s"(qs), "v"(c[s]));
            } else {
#pragma unroll
                for (int s = 0; s < 16; ++s) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(acc[s]) : "v"(qv), "v"(c[s]));
            }
            qv = qv * 1.0000001f;
        }
    }
    const long long t1 = clock64();
    float r = 0.0f;
    for (int s = 0; s < 16; ++s) r += acc[s];
    out[blockIdx.x * 512 + threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    const int blocks = 256, iters = 2000;
    float *in, *out;
    long long* cyc;
    hipMalloc(&in, 512 * 4);
    hipMalloc(&out, blocks * 512 * 4);
    hipMalloc(&cyc, blocks * 8);
    std::vector<float> h(512, 1.0f);
    hipMemcpy(in, h.data(), 512 * 4, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep)
        for (int v = 0; v < 2; ++v) {
            if (v == 0) hipLaunchKernelGGL(k<false>, dim3(blocks), dim3(512), 0, 0, in, out, cyc, iters);
            else hipLaunchKernelGGL(k<true>, dim3(blocks), dim3(512), 0, 0, in, out, cyc, iters);
            hipDeviceSynchronize();
            std::vector<long long> c(blocks);
            hipMemcpy(c.data(), cyc, blocks * 8, hipMemcpyDeviceToHost);
            double m = 0;
            for (auto x : c) m += double(x) / blocks;
            // per SIMD: 2 waves x iters x 8 x 16 fmac
            std::printf("%s: %.3f cycles per wave64 fmac per SIMD (clock64 units)\n", v ? "SGPR src0" : "VGPR src0",
                        m / (2.0 * iters * 8 * 16));
        }
    return 0;
}
