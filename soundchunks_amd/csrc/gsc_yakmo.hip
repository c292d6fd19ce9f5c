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
// 512-point block per step, with the next block's loads issued a step ahead so
// HBM latency hides under the chain.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gsc_device.h"

namespace gsc {
namespace {

__device__ __forceinline__ float fa(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fs(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ float fm(float a, float b) { return __fmul_rn(a, b); }

constexpr int kYBlock = 512;          // points per pipeline step (waves 1..8)
constexpr int kYThreads = 64 + kYBlock;  // wave 0: picks + prefix chain
constexpr int kYBits = 262144 / 32;   // chosen-point bitmap in LDS (N <= 262144)

struct YakmoShared {
    alignas(16) float ring[2][kYBlock];    // d0 of the last two blocks (chain input)
    uint32_t chosen[kYBits];
    int cursor[kMaxK];         // stable counting sort of the final assignment
    float c[32];               // current seed
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
// different grid).  Writes the four 64-point checkpoints and the new run.
__device__ __forceinline__ bool chain_step_binade(const float* __restrict__ ring, float* __restrict__ ck, int lane,
                                                  float* run_io) {
    const float run = *run_io;
    if (!(run >= 1.17549435e-38f)) return false;  // zero, negative, subnormal (or NaN)
    const int fe = __builtin_amdgcn_frexp_expf(run);  // run = f * 2^fe, f in [0.5, 1)
    const int sc = 24 - fe;                          // d/u = d * 2^sc
    const uint32_t m0 = (uint32_t)__builtin_ldexpf(run, sc);  // in [2^23, 2^24), exact
    uint32_t p[kYBlock / 64];
    bool good = true;
#pragma unroll
    for (int k = 0; k < kYBlock / 64; ++k) {
        const float t = __builtin_ldexpf(ring[k * 64 + lane], sc);  // exact unless |t| is far below 1/2
        const bool ok = __builtin_fabsf(t) < 16777216.0f && (t - __builtin_floorf(t)) != 0.5f;  // NaN: not ok
        good &= ok;
        p[k] = (uint32_t)(int)(ok ? __builtin_rintf(t) : 0.0f);
    }
#pragma unroll
    for (int k = 0; k < kYBlock / 64; ++k) p[k] = wave_incl_scan_u32(p[k], lane);
    uint32_t off = m0;
#pragma unroll
    for (int k = 0; k < kYBlock / 64; ++k) {
        const uint32_t v = off + p[k];
        // m + partial in [2^23 + 1, 2^24 - 2]: then the exact sum, within 1/2 of
        // it, lies strictly inside the binade and rounds on the grid u
        good &= (v - 8388609u) < 8388606u;
        off = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
        p[k] = off;  // the block's last partial: its checkpoint
    }
    if (__ballot(!good) != 0ull) return false;
#pragma unroll
    for (int k = 0; k < kYBlock / 64; ++k)
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
    const int nblk = (N + kYBlock - 1) / kYBlock;
    const int dt = tid - 64;  // distance thread of waves 1..4 (negative on wave 0)
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
            }
            if (lane < D) sh.c[lane] = X[(int64_t)idx * D + lane];
        }
        __syncthreads();
        const bool chain = i < K - 1;
        if (wave == 0) {
            // sequential f32 prefix over the blocks as they complete (encoder's cum[], DLL @0x180001e74)
            float run = 0.0f;
            for (int b = 0; b <= nblk; ++b) {
                if (chain && b > 0) {
                    const int base = (b - 1) * kYBlock;
                    if (base + kYBlock <= N && chain_step_binade(sh.ring[(b - 1) & 1], ckpt + (base >> 6), lane, &run))
                        goto step_done;
#pragma unroll
                    for (int k = 0; k < kYBlock / 64; ++k) {
                        const int cnt = min(64, N - (base + k * 64));
                        if (cnt == 64) {
                            // the 64 values as LDS broadcast reads into VGPRs (every lane loads
                            // the same row), then the dependent adds back to back: no VALU
                            // readlane per point on the critical chain
                            const float4* row = reinterpret_cast<const float4*>(&sh.ring[(b - 1) & 1][k * 64]);
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
                            const int v = __float_as_int(sh.ring[(b - 1) & 1][k * 64 + lane]);
                            for (int l = 0; l < cnt; ++l) run = fa(run, __int_as_float(__builtin_amdgcn_readlane(v, l)));
                        }
                        if (cnt > 0 && lane == 0) ckpt[((base + k * 64) >> 6)] = run;
                    }
                }
            step_done:
                __syncthreads();
            }
            total = run;
        } else {
            float c[D];
#pragma unroll
            for (int j = 0; j < D; ++j) c[j] = sh.c[j];
            const float cn = norm[sh.idx];
            // one pass over the points: d0/id update, block b+1 prefetched during step b
            float xv[D];
            float xn = 0.0f, dold = 0.0f;
            if (dt < N) {
#pragma unroll
                for (int j = 0; j < D; ++j) xv[j] = X[(int64_t)dt * D + j];
                xn = norm[dt];
                dold = d0[dt];
            }
            for (int b = 0; b <= nblk; ++b) {
                const int n = b * kYBlock + dt;
                if (b < nblk && n < N) {
                    float d = fa(fa(cn, xn), 0.0f);
#pragma unroll
                    for (int j = 0; j < D; ++j) d = fs(d, fm(fa(xv[j], xv[j]), c[j]));
                    float dn = dold;
                    if (i == 0 || dn > d) {
                        dn = d;
                        d0[n] = d;
                        idv[n] = i;
                    }
                    sh.ring[b & 1][dt] = dn;
                }
                const int n2 = n + kYBlock;
                if (b + 1 < nblk && n2 < N) {
#pragma unroll
                    for (int j = 0; j < D; ++j) xv[j] = X[(int64_t)n2 * D + j];
                    xn = norm[n2];
                    dold = d0[n2];
                }
                __syncthreads();
            }
        }
    }
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
