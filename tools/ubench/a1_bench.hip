// Microbenchmark of the batched scan kernel's A1 step (a1_query from
// gsc_scan.hip) in isolation: 8 waves, one block per CU, cycles per query.
#include "../../soundchunks_amd/csrc/gsc_scan.hip"
#include <cstdio>

template <int D, int LOGK, int MODE>
__global__ __launch_bounds__(512) void a1k(const float* __restrict__ in, float* __restrict__ out, int batches,
                                           unsigned long long* cyc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Scan2Shared& sh = *reinterpret_cast<Scan2Shared*>(smem);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 2 * kBatch * 16; i += blockDim.x) (&sh.q[0][0][0])[i] = in[i];
    float creg[8][D];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int d = 0; d < D; ++d) creg[s][d] = in[((tid * 8 + s) & 255) * D + d];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll 1
    for (int b = 0; b < batches; ++b) {
#pragma unroll 1
        for (int jj = 0; jj < kBatch; ++jj) {
            if (MODE == 0) {
                a1_query<D, LOGK>(sh, creg, sh.q[b & 1][jj], sh.wrec[wave][jj], wave, lane);
            } else {
                const float* qv = sh.q[b & 1][jj];
                float dv[8];
#pragma unroll
                for (int s = 0; s < 8; ++s) dv[s] = 0.0f;
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const float qd = qv[d];
#pragma unroll
                    for (int s = 0; s < 8; ++s) {
                        const float t = fsub(qd, creg[s][d]);
                        dv[s] = fadd(dv[s], fmul(t, t));
                    }
                }
                uint32_t m = 0xffffffffu;
#pragma unroll
                for (int s = 0; s < 8; ++s) m = min(m, __float_as_uint(dv[s]));
                acc ^= m;
            }
        }
        __syncthreads();
        if (MODE == 0 && lane == 0) acc ^= sh.wrec[wave][b & 31].minbits;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + tid] = __uint_as_float(acc);
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int D, int LOGK, int MODE>
void run(const char* name, float* din, float* dout, unsigned long long* dc) {
    const int batches = 500;
    const size_t shm = sizeof(Scan2Shared);
    hipFuncSetAttribute((const void*)a1k<D, LOGK, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipLaunchKernelGGL((a1k<D, LOGK, MODE>), dim3(1), dim3(512), shm, 0, din, dout, batches, dc);
    hipLaunchKernelGGL((a1k<D, LOGK, MODE>), dim3(1), dim3(512), shm, 0, din, dout, batches, dc);
    hipDeviceSynchronize();
    unsigned long long c0;
    hipMemcpy(&c0, dc, 8, hipMemcpyDeviceToHost);
    printf("%-24s %.1f cyc/query\n", name, (double)c0 / (batches * kBatch));
}

int main() {
    float *din, *dout;
    unsigned long long* dc;
    hipMalloc(&din, 8192 * 4);
    hipMalloc(&dout, 1 << 20);
    hipMalloc(&dc, 8 * 64);
    static float h[8192];
    for (int i = 0; i < 8192; ++i) h[i] = (float)((i * 37) % 101) * 0.01f;
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    run<16, 12, 0>("a1_query D16", din, dout, dc);
    run<16, 12, 1>("distances only D16", din, dout, dc);
    run<8, 12, 0>("a1_query D8", din, dout, dc);
    run<8, 12, 1>("distances only D8", din, dout, dc);
    return 0;
}
