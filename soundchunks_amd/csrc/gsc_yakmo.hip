// yakmo k-means++ seeding + seeding means (yakmo_single.dll, called by
// TFrame.Reduce at encoder.lpr:824-828 as yakmo_create(K,1,0,1,0,0,v)),
// one workgroup (9 waves) per frame.  Restated from the DLL in SURVEY.md
// App. C.1 and oracle/yakmo_oracle.c; only the means of the seeding
// assignment reach the .gsc.
//
// Per pick i the DLL walks every point once: d = ((|c|^2 + |x|^2) + 0) -
// sum_j (2 x_j) c_j (f32, dimension order), keeps the nearest seed (strict
// <) and, for i < K-1, the running f32 total cum[n] that the next pick's
// lower_bound searches.  That prefix is one sequential f32 chain per pick;
// here wave 0 runs it through 64-element registers (readlane + add) while
// the other waves compute the next block's distances.  Only every 64th cum is
// stored (a checkpoint); lower_bound replays the chain from the checkpoint
// below each probe, which reproduces cum exactly (same adds, same order) and
// therefore the DLL's probe sequence even where tiny negative d make cum
// non-monotone.
//
// Roles: wave 0 only picks and chains (the prefix, an integer prefix sum per
// binade where that is exact, see chain_step_binade); waves 1..8 compute the distances of one
// 2048-point block per step (4 points per thread), with the next block's loads issued a step ahead so
// HBM latency hides under the chain.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gsc_device.h"

namespace gsc {
namespace {

__device__ __forceinline__ float fa(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fs(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ float fm(float a, float b) { return __fmul_rn(a, b); }

constexpr int kYDist = 512;            // distance threads (waves 1..8)
constexpr int kYBlock = kYDist * 4;    // largest step (points): ring size
// points per distance thread per step (loads in flight), bounded by the VGPR
// budget of 9 waves (168): 4 rows of D = 8, 2 of D = 16, 1 of D = 32
template <int D>
constexpr int yakmo_per() {
    return 1;
}
constexpr int kYThreads = 64 + kYDist;

#ifdef GSC_STAMPS
// diagnostic phase clocks (make stamps): s_memtime deltas per role
__device__ __forceinline__ uint64_t ystamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define YST_DECL uint64_t yacc[16] = {}; uint64_t ylast = ystamp();
#define YST(k)                     \
    {                              \
        const uint64_t t_ = ystamp(); \
        yacc[k] += t_ - ylast;     \
        ylast = t_;                \
    }
#define YCNT(k) yacc[k] += 1;
#else
#define YST_DECL
#define YST(k)
#define YCNT(k)
#endif   // wave 0: picks + prefix chain
constexpr int kYBits = 262144 / 32;   // chosen-point bitmap in LDS (N <= 262144)

struct YakmoShared {
    alignas(16) float ring[2][kYBlock];    // d0 of the last two blocks (chain input)
    uint32_t chosen[kYBits];
    union {
        int cursor[kMaxK];     // stable counting sort of the final assignment
        float sdlo[kMaxK];     // picks: lower bound of |c_i - c_a|^2 per earlier seed a
    };
    float c[32];               // current seed
    float cmax;                // max |c_a|^2 over the seeds so far
    int idx;
    float total;
};

// cum[m] of the current pick, replayed from the checkpoint below m (wave 0, all lanes)
__device__ __forceinline__ float cum_at(const float* __restrict__ d0, const float* __restrict__ ckpt, int m, int lane) {
    const int blk = m >> 6;
    float run = blk > 0 ? ckpt[blk - 1] : 0.0f;
    const float v = d0[(blk << 6) + lane];  // m < N, so the block's first m - 64*blk + 1 loads are in range
    const int last = m & 63;
    for (int l = 0; l <= last; ++l) run = fa(run, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)));
    return run;
}

// Inclusive wave64 prefix sum of 32-bit integers (wrap-around arithmetic).
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t x, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

// One 256-point step of the sequential f32 prefix cum[n] = fl(cum[n-1] + d[n])
// without the dependent add chain, exact or not at all.
//
// While the running total stays in one binade [2^e, 2^(e+1)), every partial
// sum is a multiple of u = 2^(e-23): run = m*u with m in [2^23, 2^24).  Then
// fl(m*u + d) = (m + n)*u with n = round(d/u), *provided* m + d/u is not a
// tie (the even choice would depend on m) and the exact sum m + d/u stays
// inside (2^23, 2^24 - 1/2), which m + n in [2^23 + 1, 2^24 - 2] guarantees
// (the sum stays in the binade, so its rounding grid is still u).  Under
// those conditions the chain is an integer prefix sum: the d/u roundings are
// independent of each other and of the order, and the integer sums are exact.
// The step takes the fast path only when every point meets the conditions
// (no tie, |d/u| < 2^24, every partial m + n_0 + ... + n_k in range);
// otherwise it returns false and the caller adds the step point by point.
// run must be a positive normal f32 (a zero or subnormal total has a
// different grid).  Writes the NB 64-point checkpoints and the new run.
template <int NB>
__device__ __forceinline__ bool chain_step_binade(const float* __restrict__ ring, float* __restrict__ ck, int lane,
                                                  float* run_io) {
    const float run = *run_io;
    if (!(run >= 1.17549435e-38f)) return false;  // zero, negative, subnormal (or NaN)
    const int fe = __builtin_amdgcn_frexp_expf(run);  // run = f * 2^fe, f in [0.5, 1)
    const int sc = 24 - fe;                          // d/u = d * 2^sc
    const uint32_t m0 = (uint32_t)__builtin_ldexpf(run, sc);  // in [2^23, 2^24), exact
    uint32_t p[NB];
    bool good = true;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        const float t = __builtin_ldexpf(ring[k * 64 + lane], sc);  // exact unless |t| is far below 1/2
        const bool ok = __builtin_fabsf(t) < 16777216.0f && (t - __builtin_floorf(t)) != 0.5f;  // NaN: not ok
        good &= ok;
        p[k] = (uint32_t)(int)(ok ? __builtin_rintf(t) : 0.0f);
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) p[k] = wave_incl_scan_u32(p[k], lane);
    uint32_t off = m0;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        const uint32_t v = off + p[k];
        // m + partial in [2^23 + 1, 2^24 - 2]: then the exact sum, within 1/2 of
        // it, lies strictly inside the binade and rounds on the grid u
        good &= (v - 8388609u) < 8388606u;
        off = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
        p[k] = off;  // the block's last partial: its checkpoint
    }
    if (__ballot(!good) != 0ull) return false;
#pragma unroll
    for (int k = 0; k < NB; ++k)
        if (lane == 0) ck[k] = __builtin_ldexpf((float)p[k], -sc);  // exact: m < 2^24, same binade
    *run_io = __builtin_ldexpf((float)off, -sc);
    return true;
}

}  // namespace

template <int D>
__global__ __launch_bounds__(kYThreads) void yakmo_seed2_kernel(const ReduceFrame* __restrict__ frames, int nframes,
                                                                 const float* __restrict__ Xall, float* __restrict__ Call,
                                                                 float* __restrict__ f_scratch, int* __restrict__ i_scratch) {
    __shared__ YakmoShared sh;
    const int fi = blockIdx.x;
    if (fi >= nframes) return;
    const ReduceFrame fr = frames[fi];
    const int N = fr.N, K = fr.K;
    const float* __restrict__ X = Xall + fr.x_off;
    float* C = Call + fr.c_off;
    float* d0 = f_scratch + fr.n_off * 4;
    float* norm = d0 + N;
    float* ckpt = norm + N;          // N/64 + 1 checkpoints
    int* order = reinterpret_cast<int*>(ckpt + (N >> 6) + 1);  // N point indices (cluster order)
    int* idv = i_scratch + fr.n_off;  // seeding assignment
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    // yakmo point norm: norm += v*v (f32, in order) (@0x1800015cb)
    for (int n = tid; n < N; n += kYThreads) {
        const float* x = X + (int64_t)n * D;
        float s = 0.0f;
#pragma unroll
        for (int j = 0; j < D; ++j) s = fa(s, fm(x[j], x[j]));
        norm[n] = s;
    }
    for (int w = tid; w < kYBits; w += kYThreads) sh.chosen[w] = 0u;
    __syncthreads();

    uint64_t rx = 123456789ull, ry = 362436069ull, rz = 521288629ull, rw = 88675123ull;
    float total = 0.0f;
    constexpr int kYPer = yakmo_per<D>();
    constexpr int BLK = kYDist * kYPer;  // points per pipeline step
    const int nblk = (N + BLK - 1) / BLK;
    const int dt = tid - 64;  // distance thread of waves 1..4 (negative on wave 0)
    YST_DECL
    for (int i = 0; i < K; ++i) {
        // ---- pick (wave 0; the RNG runs redundantly in every thread)
        const uint64_t t = rx ^ (rx << 11);
        rx = ry;
        ry = rz;
        rz = rw;
        rw = rw ^ (rw >> 19) ^ t ^ (t >> 8);
        const float r = (float)((double)rw * 5.42101086242752217e-20);  // f32(f64(w) * 2^-64)
        if (wave == 0) {
            uint32_t idx;
            if (i == 0) {
                idx = (uint32_t)(int64_t)floorf(fm(r, (float)N));
            } else {
                // std::lower_bound(cum, cum + N, r * total): r*total > cum[mid] moves right
                const float target = fm(r, total);
                int first = 0, count = N;
                while (count > 0) {
                    const int half = count >> 1;
                    const int mid = first + half;
                    if (target > cum_at(d0, ckpt, mid, lane)) {
                        first = mid + 1;
                        count -= half + 1;
                    } else {
                        count = half;
                    }
                }
                idx = (uint32_t)(int64_t)(float)first;
            }
            // collision walk (@0x180001b20) and clamp (@0x180001c50)
            while (idx < (uint32_t)N && ((sh.chosen[idx >> 5] >> (idx & 31)) & 1u))
                idx = (idx < (uint32_t)(N - 1)) ? idx + 1 : 0u;
            if (idx >= (uint32_t)N) idx = (uint32_t)(N - 1);
            if (lane == 0) {
                sh.chosen[idx >> 5] |= 1u << (idx & 31);
                sh.idx = (int)idx;
                sh.cmax = i == 0 ? norm[idx] : fmaxf(sh.cmax, norm[idx]);
            }
            if (lane < D) {
                const float v = X[(int64_t)idx * D + lane];
                sh.c[lane] = v;
                C[(int64_t)i * D + lane] = v;  // the seeds (C is overwritten by the means at the end)
            }
            YST(0)
        }
        __syncthreads();
        const bool chain = i < K - 1;
        if (wave == 0) {
            YST(3)
            __syncthreads();  // the distance waves' seed-distance table
            YST(3)
            // sequential f32 prefix over the blocks as they complete (encoder's cum[], DLL @0x180001e74)
            float run = 0.0f;
            for (int b = 0; b <= nblk; ++b) {
                if (chain && b > 0) {
                    const int base = (b - 1) * BLK;
                    const float* rg = sh.ring[(b - 1) & 1];
                    if (base + BLK <= N && chain_step_binade<BLK / 64>(rg, ckpt + (base >> 6), lane, &run)) {
                        YST(1) YCNT(4)
                        __syncthreads();
                        YST(3)
                        continue;
                    }
                    for (int k = 0; k < BLK / 64; ++k) {
                        const int cnt = min(64, N - (base + k * 64));
                        if (cnt <= 0) break;
                        if (cnt == 64) {
                            // the 64 values as LDS broadcast reads into VGPRs (every lane loads
                            // the same row), then the dependent adds back to back: no VALU
                            // readlane per point on the critical chain
                            const float4* row = reinterpret_cast<const float4*>(&rg[k * 64]);
                            float4 sv[16];
#pragma unroll
                            for (int l = 0; l < 16; ++l) sv[l] = row[l];
#pragma unroll
                            for (int l = 0; l < 16; ++l) {
                                run = fa(run, sv[l].x);
                                run = fa(run, sv[l].y);
                                run = fa(run, sv[l].z);
                                run = fa(run, sv[l].w);
                            }
                        } else {
                            const int v = __float_as_int(rg[k * 64 + lane]);
                            for (int l = 0; l < cnt; ++l) run = fa(run, __int_as_float(__builtin_amdgcn_readlane(v, l)));
                        }
                        if (lane == 0) ckpt[((base + k * 64) >> 6)] = run;
                    }
                    YST(2) YCNT(5)
                }
                __syncthreads();
                YST(3)
            }
            total = run;
        } else {
            float c[D];
#pragma unroll
            for (int j = 0; j < D; ++j) c[j] = sh.c[j];
            const float cn = norm[sh.idx];
            const float cmax = sh.cmax;
            // Seed-distance table: sdlo[a] <= |c_i - c_a|^2 (the f32 sum of squared
            // differences, lowered by 2^-16 relative to cover its rounding).
            for (int a = dt; a < i; a += kYDist) {
                float s2 = 0.0f;
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    const float t = fs(C[(int64_t)a * D + j], c[j]);
                    s2 = fa(s2, fm(t, t));
                }
                sh.sdlo[a] = fm(s2, 0.99998474f);
            }
            YST(8)
            __syncthreads();
            YST(8)
            // Elkan skip: with E = (|x|^2 + cmax) 2^-16 >= the rounding error of any of the
            // DLL's expanded-form distances from x (< 80 u (|x|^2 + |c|^2)), the computed
            // d0 = d(x, c_a) and d(x, c_i) are within E of the true squares, so
            // |c_i - c_a| >= 2 sqrt(max(d0, 0) + E) implies d(x, c_i) >= d0: no strict
            // improvement, and the point's X row need not be read for this pick.
            auto skip_of = [&](float dold, float xn, int a) -> bool {
                if (i == 0) return false;
                const float e = fm(fa(xn, cmax), 1.52587891e-05f);
                const float need = fm(fm(fa(fmaxf(dold, 0.0f), e), 4.0f), 1.00000381f);
                return sh.sdlo[a] >= need;
            };
            // one pass over the points: d0/id update; block b+1's X rows (when not
            // skipped) and block b+2's d0/|x|^2/id are loaded during step b.  Each
            // thread owns kYPer points per block (kYDist apart, coalesced).
            float xv[kYPer][D];
            float xn[kYPer], dold[kYPer], xn_n[kYPer], dold_n[kYPer];
            bool skip[kYPer];
            int a_n[kYPer];
#pragma unroll
            for (int q = 0; q < kYPer; ++q) {
                const int n0 = q * kYDist + dt, n1 = n0 + BLK;
                xn[q] = 0.0f;
                dold[q] = 0.0f;
                skip[q] = true;
                if (n0 < N) {
                    xn[q] = norm[n0];
                    dold[q] = d0[n0];
                    skip[q] = skip_of(dold[q], xn[q], i == 0 ? 0 : idv[n0]);
                    if (!skip[q]) {
#pragma unroll
                        for (int j = 0; j < D; ++j) xv[q][j] = X[(int64_t)n0 * D + j];
                    }
                }
                xn_n[q] = 0.0f;
                dold_n[q] = 0.0f;
                a_n[q] = 0;
                if (n1 < N) {
                    xn_n[q] = norm[n1];
                    dold_n[q] = d0[n1];
                    a_n[q] = i == 0 ? 0 : idv[n1];
                }
            }
            for (int b = 0; b <= nblk; ++b) {
#pragma unroll
                for (int q = 0; q < kYPer; ++q) {
                    const int n = b * BLK + q * kYDist + dt;
                    if (b < nblk && n < N) {
                        float dn = dold[q];
                        if (!skip[q]) {
                            float d = fa(fa(cn, xn[q]), 0.0f);
#pragma unroll
                            for (int j = 0; j < D; ++j) d = fs(d, fm(fa(xv[q][j], xv[q][j]), c[j]));
                            if (i == 0 || dn > d) {
                                dn = d;
                                d0[n] = d;
                                idv[n] = i;
                            }
                        }
                        sh.ring[b & 1][q * kYDist + dt] = dn;
                    }
                }
#pragma unroll
                for (int q = 0; q < kYPer; ++q) {
                    const int n2 = (b + 1) * BLK + q * kYDist + dt;
                    if (b + 1 < nblk && n2 < N) {
                        xn[q] = xn_n[q];
                        dold[q] = dold_n[q];
                        skip[q] = skip_of(dold[q], xn[q], a_n[q]);
                        if (!skip[q]) {
#pragma unroll
                            for (int j = 0; j < D; ++j) xv[q][j] = X[(int64_t)n2 * D + j];
                        }
                        const int n3 = n2 + BLK;
                        if (b + 2 < nblk && n3 < N) {
                            xn_n[q] = norm[n3];
                            dold_n[q] = d0[n3];
                            a_n[q] = i == 0 ? 0 : idv[n3];
                        }
                    }
                }
                YST(9)
                __syncthreads();
                YST(10)
            }
        }
    }
#ifdef GSC_STAMPS
    if (tid == 0 || tid == 64) {
        uint64_t* ys = const_cast<ReduceFrame*>(frames)[fi].ystamps;
        for (int k = 0; k < 16; ++k)
            if ((tid == 0) == (k < 8)) ys[k] = yacc[k];
    }
#endif
    // ---- means of the seeding assignment (@0x180002290): c = f32(sum in point order) / f32(count)
    int* counts = i_scratch + fr.k_off;
    for (int k = tid; k < K; k += kYThreads) sh.cursor[k] = 0;
    __syncthreads();
    for (int n = tid; n < N; n += kYThreads) atomicAdd(&sh.cursor[idv[n]], 1);
    __syncthreads();
    if (tid == 0) {  // exclusive prefix of the counts
        int acc = 0;
        for (int k = 0; k < K; ++k) {
            const int v = sh.cursor[k];
            counts[k] = v;
            sh.cursor[k] = acc;
            acc += v;
        }
    }
    __syncthreads();
    if (wave == 0) {  // stable placement: points in index order per cluster
        for (int base = 0; base < N; base += 64) {
            const int n = base + lane;
            const int id = n < N ? idv[n] : -1;
            const int cnt = min(64, N - base);
            for (int l = 0; l < cnt; ++l) {
                const int cl = __builtin_amdgcn_readlane(id, l);
                if (lane == 0) order[sh.cursor[cl]++] = base + l;
            }
        }
    }
    __syncthreads();
    for (int k = tid; k < K; k += kYThreads) {
        const int cnt = counts[k];
        const int start = sh.cursor[k] - cnt;
        float s[D];
#pragma unroll
        for (int j = 0; j < D; ++j) s[j] = 0.0f;
        for (int m = 0; m < cnt; ++m) {
            const float* x = X + (int64_t)order[start + m] * D;
#pragma unroll
            for (int j = 0; j < D; ++j) s[j] = fa(s[j], x[j]);
        }
        const float fc = (float)(int64_t)(uint32_t)cnt;
#pragma unroll
        for (int j = 0; j < D; ++j) C[(int64_t)k * D + j] = s[j] / fc;  // IEEE division; 0/0 = NaN like the DLL
    }
}

}  // namespace gsc

using namespace gsc;

extern "C" hipError_t gsc_launch_yakmo(int D, const ReduceFrame* frames, int nframes, const float* X, float* C,
                                       float* fs, int* is, uint32_t* /*bits*/, hipStream_t st) {
    dim3 grid(nframes), block(kYThreads);
    switch (D) {
    case 8: hipLaunchKernelGGL(yakmo_seed2_kernel<8>, grid, block, 0, st, frames, nframes, X, C, fs, is); break;
    case 16: hipLaunchKernelGGL(yakmo_seed2_kernel<16>, grid, block, 0, st, frames, nframes, X, C, fs, is); break;
    case 32: hipLaunchKernelGGL(yakmo_seed2_kernel<32>, grid, block, 0, st, frames, nframes, X, C, fs, is); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
