// Microbenchmark of the batched scan kernel's A1 step in isolation: 8 waves,
// one block per CU, ticks (s_memtime) per query, plus the tick rate from
// hipEvents so ticks convert to ns.
//   MODE 0  a1_query from gsc_scan.hip (the kernel's A1)
//   MODE 1  distances + lane min only (the floor)
//   MODE 2  min-tree with v_permlane16/32_swap for the two widest levels
//           (no ds_swizzle, no readlane round trip)
#include "../../soundchunks_amd/csrc/gsc_scan.hip"
#include <cstdio>

namespace gsc {
template <int LOGK>
__device__ __forceinline__ void a1_reduce_pl(const float (&dv)[8], WaveRec& rec, int wave, int lane) {
    constexpr int K = 1 << LOGK;
    const int p0 = (wave * 64 + lane) * 8;
    uint32_t b[8];
    const bool has = LOGK >= 9 || p0 < K;
#pragma unroll
    for (int s = 0; s < 8; ++s) b[s] = has ? __float_as_uint(dv[s]) : 0xFFFFFFFFu;
    const uint32_t m01 = min(b[0], b[1]), m23 = min(b[2], b[3]), m45 = min(b[4], b[5]), m67 = min(b[6], b[7]);
    const uint32_t m03 = min(m01, m23), m47 = min(m45, m67);
    const uint32_t lmin = min(m03, m47);
    uint32_t v = lmin;
    const uint32_t sl0 = partner<0>(v);
    v = min(v, sl0);
    const uint32_t sl1 = partner<1>(v);
    v = min(v, sl1);
    const uint32_t sl2 = partner<2>(v);
    v = min(v, sl2);
    const uint32_t sl3 = partner<3>(v);
    v = min(v, sl3);
    const auto p16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    const uint32_t sl4 = (lane & 16) ? p16[0] : p16[1];
    v = min(p16[0], p16[1]);
    const auto p32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    const uint32_t sl5 = (lane & 32) ? p32[0] : p32[1];
    const uint32_t wmin = min(p32[0], p32[1]);
    const uint64_t m = __ballot(lmin == wmin);
    const int L = __ffsll((long long)m) - 1;
    if (lane == L) {
        int ls = 7, lc = 0;
#pragma unroll
        for (int s = 7; s >= 0; --s) {
            const bool e = b[s] == lmin;
            lc += e ? 1 : 0;
            ls = e ? s : ls;
        }
        const uint32_t pa = (ls & 4) ? ((ls & 2) ? b[6] : b[4]) : ((ls & 2) ? b[2] : b[0]);
        const uint32_t pb = (ls & 4) ? ((ls & 2) ? b[7] : b[5]) : ((ls & 2) ? b[3] : b[1]);
        rec.minbits = wmin;
        rec.tie = (__popcll(m) > 1 || lc > 1) ? 1 : 0;
        rec.pos = p0 + ls;
        rec.sib[0] = sl0;
        rec.sib[1] = sl1;
        rec.sib[2] = sl2;
        rec.sib[3] = sl3;
        rec.sib[4] = sl4;
        rec.sib[5] = sl5;
        rec.sib[6] = (ls & 1) ? pa : pb;
        rec.sib[7] = (ls & 4) ? ((ls & 2) ? m45 : m67) : ((ls & 2) ? m01 : m23);
        rec.sib[8] = (ls & 4) ? m03 : m47;
    }
}
}  // namespace gsc

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
            const float* qv = sh.q[b & 1][jj];
            float dv[8];
            a1_dist<D>(creg, qv, dv);
            if (MODE == 0) {
                a1_reduce<LOGK>(dv, sh.wrec[wave][jj], wave, lane);
            } else if (MODE == 2) {
                a1_reduce_pl<LOGK>(dv, sh.wrec[wave][jj], wave, lane);
            } else {
                uint32_t m = 0xffffffffu;
#pragma unroll
                for (int s = 0; s < 8; ++s) m = min(m, __float_as_uint(dv[s]));
                acc ^= m;
            }
        }
        __syncthreads();
        if (MODE != 1 && lane == 0) acc ^= sh.wrec[wave][b & 31].minbits ^ sh.wrec[wave][b & 31].sib[5];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + tid] = __uint_as_float(acc);
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int D, int LOGK, int MODE>
void run(const char* name, float* din, float* dout, unsigned long long* dc, int nblk) {
    const int batches = 500;
    const size_t shm = sizeof(Scan2Shared);
    hipFuncSetAttribute((const void*)a1k<D, LOGK, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipLaunchKernelGGL((a1k<D, LOGK, MODE>), dim3(nblk), dim3(512), shm, 0, din, dout, batches, dc);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((a1k<D, LOGK, MODE>), dim3(nblk), dim3(512), shm, 0, din, dout, batches, dc);
    hipEventRecord(e1, 0);
    hipDeviceSynchronize();
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c0;
    hipMemcpy(&c0, dc, 8, hipMemcpyDeviceToHost);
    const double q = (double)batches * kBatch;
    printf("%-28s blocks %3d  %.1f ticks/query  %.1f ns/query  (tick rate %.0f MHz)\n", name, nblk, (double)c0 / q,
           ms * 1e6 / q, (double)c0 / (ms * 1e3));
}

int main() {
    float *din, *dout;
    unsigned long long* dc;
    hipMalloc(&din, 8192 * 4);
    hipMalloc(&dout, 1 << 22);
    hipMalloc(&dc, 8 * 512);
    static float h[8192];
    for (int i = 0; i < 8192; ++i) h[i] = (float)((i * 37) % 101) * 0.01f;
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    for (int nb : {1, 256}) {
        run<16, 12, 0>("a1_query D16", din, dout, dc, nb);
        run<16, 12, 2>("a1 permlane D16", din, dout, dc, nb);
        run<16, 12, 1>("distances only D16", din, dout, dc, nb);
    }
    run<8, 12, 0>("a1_query D8", din, dout, dc, 1);
    run<8, 12, 2>("a1 permlane D8", din, dout, dc, 1);
    run<8, 12, 1>("distances only D8", din, dout, dc, 1);
    return 0;
}
