// yakmo k-means++ seeding + seeding means (yakmo_single.dll, called by
// TFrame.Reduce at encoder.lpr:824-828 as yakmo_create(K,1,0,1,0,0,v)),
// one workgroup (9 waves) per frame.  Restated from the DLL in SURVEY.md
// App. C.1 and oracle/yakmo_oracle.c; only the means of the seeding
// assignment reach the .gsc.
//
// Per pick i the DLL walks every point once: d = ((|c|^2 + |x|^2) + 0) -
// sum_j (2 x_j) c_j (f32, dimension order), keeps the nearest seed (strict
// <) and, for i < K-1, the running f32 total cum[n] that the next pick's
// lower_bound searches.  That prefix is one sequential f32 chain per pick.
//
// Roles: wave 0 picks and chains; 8 distance waves compute one 1024-point
// block per step (two points per thread; 512 at D = 32), d0 and seed ids
// prefetched three steps ahead and the X rows of points that the Elkan bound
// cannot skip one step ahead; three more waves only keep the barriers, so the
// chain issues alone on its SIMD.
// The chain turns each run of whole 64-point blocks into one integer prefix
// sum while the total stays in one binade (chain_fast: exact, or the blocks
// are added one by one), and keeps per 64-point block the checkpoint cum and
// the block's min / max in LDS.  The next pick's lower_bound then finds its
// block from the maxima and proves from the minima that the DLL's binary
// search cannot end anywhere else (pick_lower_bound), replaying one block;
// where it cannot prove that, it replays the DLL's probe sequence.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gsc_device.h"

namespace gsc {
namespace {

__device__ __forceinline__ float fa(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fs(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ float fm(float a, float b) { return __fmul_rn(a, b); }

constexpr int kYDist = 512;            // distance threads (8 waves)
// points per distance thread per step (kYDist apart): two at D <= 16, one at
// D = 32 (VGPR budget)
template <int D>
constexpr int yakmo_pts() {
    return D == 32 ? 1 : 2;
}
constexpr int kYBlock = kYDist * 2;    // ring capacity: points per step (largest)
// 12 waves, 3 per SIMD: wave 0 picks and chains; waves 4, 8 and 11 only keep
// the barriers, so SIMD 0 issues the chain alone; the other 8 compute distances
constexpr int kYThreads = 768;
__device__ __forceinline__ bool yakmo_idle_wave(int w) { return w == 4 || w == 8 || w == 11; }
// distance thread index of a distance wave's lane
__device__ __forceinline__ int yakmo_dist_index(int w, int lane) { return (w - 1 - w / 4) * 64 + lane; }
constexpr int kYMaxLds = 262144;      // frames up to this many points keep the yakmo state in LDS
constexpr int kYBits = kYMaxLds / 32;  // chosen-point bitmap in LDS
#ifndef GSC_YAKMO_XD
#define GSC_YAKMO_XD 1
#endif
constexpr int kYXD = GSC_YAKMO_XD;    // X-row look-ahead in steps
constexpr int kYPre = kYXD == 1 ? 3 : 4;  // d0 / seed-id prefetch depth (steps), a multiple of kYXD

#ifdef GSC_STAMPS
// diagnostic phase clocks (make stamps): s_memtime deltas per role
__device__ __forceinline__ uint64_t ystamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
// a delta that comes out negative (s_memtime read backwards once: round 5's
// "slow" slot carried one frame's wrapped sum, 2^64 / (frames x picks)) is
// not added but counted in slot 6 (wave 0) / 14 (distance waves)
#define YST_DECL uint64_t yacc[16] = {}; uint64_t ylast = ystamp();
#define YST(k)                                      \
    {                                               \
        const uint64_t t_ = ystamp();               \
        const int64_t d_ = (int64_t)(t_ - ylast);   \
        if (d_ >= 0)                                \
            yacc[k] += (uint64_t)d_;                \
        else                                        \
            yacc[(k) < 8 ? 6 : 14] += 1;            \
        ylast = t_;                                 \
    }
#define YCNT(k) yacc[k] += 1;
#else
#define YST_DECL
#define YST(k)
#define YCNT(k)
#endif

struct YakmoShared {
    alignas(16) float ring[2][kYBlock];    // d0 of the last two blocks (chain input)
    uint32_t chosen[kYBits];
    union {
        int cursor[kMaxK];     // stable counting sort of the final assignment
        float sdlo[kMaxK];     // picks: lower bound of |c_i - c_a|^2 per earlier seed a
    };
    float c[32];               // current seed
    float cn;                  // its |c|^2
    float cmax;                // max |c_a|^2 over the seeds so far
    float xmax;                // max |x|^2 over the frame's points
};
// dynamic LDS after YakmoShared, per 64-point block g of the current pick's
// prefix cum[]: ck[g] = cum at the block's last point, bmn/bmx[g] = min/max of
// the block's cum values

// Barrier for LDS hand-offs only: the global loads in flight (the distance
// waves' prefetch) stay in flight, which __syncthreads' full fence would drain.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// step barrier: LDS only, except the last step of a pick, which also orders
// the pick's global d0 / seed-id / seed stores before the next pick reads them
__device__ __forceinline__ void step_barrier(bool last) {
    if (last)
        __syncthreads();
    else
        lds_barrier();
}

__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// cum[m] of the current pick, replayed from the checkpoint below m (wave 0, all lanes)
__device__ __forceinline__ float cum_at(const float* __restrict__ d0, const float* ck, int m, int lane) {
    const int blk = m >> 6;
    float run = blk > 0 ? ck[blk - 1] : 0.0f;
    const float v = d0[(blk << 6) + lane];  // m < N, so the block's first m - 64*blk + 1 loads are in range
    const int last = m & 63;
    for (int l = 0; l <= last; ++l) run = fa(run, readlane_f(v, l));
    return run;
}

// Inclusive wave64 prefix sum of 32-bit integers (wrap-around) by DPP:
// row_shr 1/2/4/8 inside each row of 16, then row_bcast:15 / row_bcast:31
// carry the row totals into the rows above.
__device__ __forceinline__ uint32_t wave_scan_u32(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// f32 -> i32 as v_cvt_i32_f32 does it: saturating, NaN -> 0 (a C++ cast of
// an out-of-range value would be undefined)
__device__ __forceinline__ int cvt_sat_i32(float x) {
    int r;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// Inclusive wave64 running max of non-negative integers (same DPP pattern)
__device__ __forceinline__ int wave_max_scan(int x) {
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false));
    return x;
}

// min / max over the 8 lanes of an aligned lane octet (DPP: quad_perm
// [1,0,3,2], [2,3,0,1], then row_half_mirror across the two quads)
__device__ __forceinline__ uint32_t oct_min_u32(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xb1, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4e, 0xf, 0xf, false));
    return min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false));
}
__device__ __forceinline__ uint32_t oct_max_u32(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xb1, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4e, 0xf, 0xf, false));
    return max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false));
}

// The sequential f32 prefix cum[n] = fl(cum[n-1] + d[n]) over whole 64-point
// blocks without the dependent add chain, exact or not at all.
//
// While the running total stays in one binade [2^e, 2^(e+1)), every partial
// sum is a multiple of u = 2^(e-23): run = m*u with m in [2^23, 2^24).  Then
// fl(m*u + d) = (m + n)*u with n = round(d/u), *provided* m + d/u is not a
// tie (the even choice would depend on m) and the exact sum m + d/u stays
// inside (2^23, 2^24 - 1/2), which m + n in [2^23 + 1, 2^24 - 2] guarantees
// (the sum stays in the binade, so its rounding grid is still u).  Under
// those conditions the chain is an integer prefix sum: the d/u roundings are
// independent of each other and of the order, and the integer sums are exact.
//
// Points s .. s + 64 nbk - 1 of the ring (nbk <= 64 PPL / 64 blocks, s a
// multiple of 64); lane l takes PPL consecutive points: one local prefix, one
// wave scan.  The blocks before the first lane holding a point that breaks a
// condition (tie, |d/u| >= 2^24, NaN, a partial out of range) are accepted:
// their checkpoints and min/max are written (global block index g0 + k) and
// *run_io moves to the last accepted partial.  Returns the accepted block
// count.  |run| must be at least 2^-100, so that 2^sc is a normal f32 and
// d * 2^sc is exact wherever it matters (a d/u far below 1/2 may round: it
// still rounds to 0, no tie); at run == 0 the leading blocks whose points are
// all +-0 are accepted (fl(+0 + +-0) = +0: every partial stays +0).
//
// The check is per lane, on the lane's partials' min and max: lanes before
// the first bad lane have every partial in range, so the first bad lane's
// base is its exact predecessor partial; there a point with a tie or NaN
// fails |t - rint(t)| < 1/2, and the first partial out of range is out of
// range mod 2^32 as well (|n| < 2^24 + 2^23 would be needed to come back),
// so the min or the max of the lane's base + partials (exact mod 2^32, as
// int32) leaves [2^23 + 1, 2^24 - 2].
template <int PPL>
__device__ __forceinline__ int chain_fast(const float* __restrict__ ring, int s, int nbk, int lane, float* run_io,
                                          float* ck, float* bmn, float* bmx, int g0) {
    static_assert(PPL == 8 || PPL == 16, "8 or 16 points per lane");
    constexpr int LPB = 64 / PPL;  // lanes per 64-point block
    const float run = *run_io;
    const bool act = lane < nbk * LPB;
    float v[PPL];
    if (act) {
#pragma unroll
        for (int h = 0; h < PPL / 4; ++h) {
            const float4 a = *reinterpret_cast<const float4*>(&ring[s + PPL * lane + 4 * h]);
            v[4 * h] = a.x, v[4 * h + 1] = a.y, v[4 * h + 2] = a.z, v[4 * h + 3] = a.w;
        }
    } else {
#pragma unroll
        for (int e = 0; e < PPL; ++e) v[e] = 0.0f;
    }
    // a negative run: the same on the negated points (round-to-nearest-even
    // is odd-symmetric), partials m*u with m in [2^23, 2^24) from -run
    const float arun = __builtin_fabsf(run);
    if (!(arun >= 7.88860905e-31f)) {  // below 2^-100 in magnitude, zero (or NaN)
        if (run != 0.0f) return 0;
        bool nz = false;
#pragma unroll
        for (int e = 0; e < PPL; ++e) nz = nz || v[e] != 0.0f;  // NaN: != 0
        const uint64_t bz = __ballot(act && nz);
        const int k = bz ? min(nbk, __builtin_ctzll(bz) / LPB) : nbk;
        const int blk = lane / LPB;
        if (blk < k) {
            if ((lane % LPB) == 0) bmn[g0 + blk] = bmx[g0 + blk] = 0.0f;
            if ((lane % LPB) == LPB - 1) ck[g0 + blk] = 0.0f;
        }
        return k;  // run stays +0
    }
    const int fe = __builtin_amdgcn_frexp_expf(arun);  // |run| = f * 2^fe, f in [0.5, 1)
    const int sc = 24 - fe;                           // d/u = d * 2^sc, sc <= 124
    const float sgn = run < 0.0f ? -1.0f : 1.0f;
    const float scale = sgn * __builtin_ldexpf(1.0f, sc), unscale = sgn * __builtin_ldexpf(1.0f, -sc);
    const uint32_t m0 = (uint32_t)(run * scale);  // in [2^23, 2^24), exact
    int n[PPL];
    bool ok = true;
#pragma unroll
    for (int e = 0; e < PPL; ++e) {
        const float t = v[e] * scale;
        const float r = __builtin_rintf(t);
        ok = ok && __builtin_fabsf(t - r) < 0.5f;  // ties, NaN and infinities fail
        n[e] = cvt_sat_i32(r);  // |t| >= 2^24 fails the range check
    }
    // lane total as a tree, then the lane's partials from its base
    uint32_t acc = 0;
#pragma unroll
    for (int e = 0; e < PPL; ++e) acc += (uint32_t)n[e];
    const uint32_t p0 = m0 + (wave_scan_u32(acc) - acc);
    uint32_t p = p0;
    int mn = 0x7fffffff, mx = -0x7fffffff - 1;
#pragma unroll
    for (int e = 0; e < PPL; ++e) {
        p += (uint32_t)n[e];
        mn = min(mn, (int)p);
        mx = max(mx, (int)p);
    }
    const uint64_t bl = __ballot(act && !(ok && mn >= 8388609 && mx <= 16777214));
    int k = bl ? min(nbk, __builtin_ctzll(bl) / LPB) : nbk;
#ifndef GSC_YAKMO_NO_TIES
    // (only when the first failing lane itself holds a tie, NaN or infinity:
    // a lane that fails on range alone has no tie, and the lanes before it
    // none either, so resolving ties cannot move k -- a binade crossing)
    if (k < nbk && __builtin_amdgcn_readlane((int)ok, __builtin_ctzll(bl)) == 0) {
        // A tie t = j + 1/2 rounds to the even one of m + j, m + j + 1, with m
        // the exact partial before it: rint(t) + c, c = 0 if m is even, else
        // +1 (t - rint(t) = +1/2) or -1.  Each c != 0 flips the parity of all
        // later partials, so the parity of the adjustments made up to and
        // including tie i equals the parity b_i of the unadjusted (rint)
        // partial at tie i, and c_i != 0 exactly when b_i != b_(i-1) (b_0 = 0).
        // Two passes over the points, reloaded and re-rounded one at a time
        // (nothing stays live across the first pass): the lanes' last tie
        // parities, then the adjusted partials; t is clamped to 2^25 there,
        // so the lane-relative partials stay below 2^30 and their min / max
        // plus the lane base are exact.
        const float4* row = reinterpret_cast<const float4*>(&ring[s + PPL * lane]);
        uint32_t q = p0;
        int key = 0;  // 2 lane + 1 + parity of the lane's last tie, 0: none
#pragma unroll
        for (int h = 0; h < PPL / 4; ++h) {
            const float4 a = act ? row[h] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            const float x4[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
            for (int l = 0; l < 4; ++l) {
                const float t = x4[l] * scale;
                const float r = __builtin_rintf(__builtin_amdgcn_fmed3f(t, -33554432.0f, 33554432.0f));
                q += (uint32_t)cvt_sat_i32(r);
                key = __builtin_fabsf(t - r) == 0.5f ? 2 * lane + 1 + (int)(q & 1u) : key;
            }
        }
        if (__ballot(act && key != 0)) {
            const int prev = __builtin_amdgcn_update_dpp(0, wave_max_scan(key), 0x138, 0xf, 0xf, false);  // wave_shr:1
            uint32_t bprev = prev ? (uint32_t)(prev - 1) & 1u : 0u;
            bool okt = true;
            int rel = 0, rmn = 0x7fffffff, rmx = -0x7fffffff - 1, csum = 0;
            q = p0;
#pragma unroll
            for (int h = 0; h < PPL / 4; ++h) {
                const float4 a = act ? row[h] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                const float x4[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
                for (int l = 0; l < 4; ++l) {
                    const float t = x4[l] * scale;
                    const float r = __builtin_rintf(__builtin_amdgcn_fmed3f(t, -33554432.0f, 33554432.0f));
                    const float dlt = t - r;
                    const int ni = cvt_sat_i32(r);
                    okt = okt && __builtin_fabsf(dlt) <= 0.5f;  // NaN and |t| > 2^25 fail
                    q += (uint32_t)ni;
                    const bool tie = __builtin_fabsf(dlt) == 0.5f;
                    const uint32_t b = q & 1u;
                    const int c = (tie && b != bprev) ? (dlt < 0.0f ? -1 : 1) : 0;
                    bprev = tie ? b : bprev;
                    csum += c;
                    rel += ni + c;
                    rmn = min(rmn, rel);
                    rmx = max(rmx, rel);
                }
            }
            const uint32_t base = p0 + (wave_scan_u32((uint32_t)csum) - (uint32_t)csum);
            mn = (int)(base + (uint32_t)rmn);
            mx = (int)(base + (uint32_t)rmx);
            p = base + (uint32_t)rel;
            const uint64_t b2 = __ballot(act && !(okt && mn >= 8388609 && mx <= 16777214));
            k = b2 ? min(nbk, __builtin_ctzll(b2) / LPB) : nbk;
        }
    }
#endif
    if (k == 0) return 0;
    // accepted lanes: in range, so integer order is the partials' order
    if constexpr (PPL == 8) {
        mn = (int)oct_min_u32((uint32_t)mn);
        mx = (int)oct_max_u32((uint32_t)mx);
    } else {
        mn = min(mn, __builtin_amdgcn_mov_dpp(mn, 0xb1, 0xf, 0xf, false));
        mx = max(mx, __builtin_amdgcn_mov_dpp(mx, 0xb1, 0xf, 0xf, false));
        mn = min(mn, __builtin_amdgcn_mov_dpp(mn, 0x4e, 0xf, 0xf, false));
        mx = max(mx, __builtin_amdgcn_mov_dpp(mx, 0x4e, 0xf, 0xf, false));
    }
    const int blk = lane / LPB;
    if (blk < k) {
        if ((lane % LPB) == 0) {
            const float a = (float)mn * unscale, b = (float)mx * unscale;  // exact: < 2^24, same binade
            bmn[g0 + blk] = fminf(a, b);  // (swapped for a negative run)
            bmx[g0 + blk] = fmaxf(a, b);
        }
        if ((lane % LPB) == LPB - 1) ck[g0 + blk] = (float)p * unscale;
    }
    *run_io = (float)(uint32_t)__builtin_amdgcn_readlane((int)p, LPB * k - 1) * unscale;
    return k;
}

// c <= 64 points of the ring from s added one by one (the reference's chain)
__device__ __forceinline__ void chain_seq(const float* __restrict__ ring, int s, int c, int lane, float* run_io,
                                          float* ck, float* bmn, float* bmx, int g) {
    float run = *run_io, mn = 3.4028235e38f, mx = -3.4028235e38f;
    if (c == 64) {
        // the values as LDS broadcast reads into VGPRs (every lane loads the
        // same row, 16 at a time, the next 16 in flight), then the dependent
        // adds back to back
        const float4* row = reinterpret_cast<const float4*>(&ring[s]);
        float4 sv[4], nx[4];
#pragma unroll
        for (int l = 0; l < 4; ++l) sv[l] = row[l];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            if (h < 3) {
#pragma unroll
                for (int l = 0; l < 4; ++l) nx[l] = row[4 * (h + 1) + l];
            }
#pragma unroll
            for (int l = 0; l < 4; ++l) {
                run = fa(run, sv[l].x);
                mn = fminf(mn, run), mx = fmaxf(mx, run);
                run = fa(run, sv[l].y);
                mn = fminf(mn, run), mx = fmaxf(mx, run);
                run = fa(run, sv[l].z);
                mn = fminf(mn, run), mx = fmaxf(mx, run);
                run = fa(run, sv[l].w);
                mn = fminf(mn, run), mx = fmaxf(mx, run);
            }
#pragma unroll
            for (int l = 0; l < 4; ++l) sv[l] = nx[l];
        }
    } else {
        const float v = lane < c ? ring[s + lane] : 0.0f;
        for (int l = 0; l < c; ++l) {
            run = fa(run, readlane_f(v, l));
            mn = fminf(mn, run), mx = fmaxf(mx, run);
        }
    }
    if (lane == 0) {
        ck[g] = run;
        bmn[g] = mn;
        bmx[g] = mx;
    }
    *run_io = run;
}

// std::lower_bound(cum, cum + N, target) of the DLL's pick (@0x180001b20).
// The probe sequence matters only where cum is not partitioned by target
// (cum dips when a d0 is negative, e.g. a seed's own expanded-form distance).
// If every cum before i* = the first index with cum >= target is below target
// (true by definition) and every cum from i* on is >= target, any binary
// search returns i*.  i*'s block is the first whose max reaches target; the
// blocks after it are checked by their minima, i*'s own block by replaying it
// from its checkpoint.  Otherwise (or with a non-finite total) the DLL's probe
// sequence is replayed exactly.
__device__ int pick_lower_bound(float target, float total, int N, const float* ck, const float* bmn, const float* bmx,
                                const float* __restrict__ d0, int lane) {
    const int nb = (N + 63) >> 6;
    if (__builtin_isfinite(total)) {
        int bstar = -1;
        float suf = 3.4028235e38f;
        for (int c0 = 0; c0 < nb; c0 += 64) {
            const int g = c0 + lane;
            const bool valid = g < nb;
            if (bstar < 0) {
                const uint64_t m = __ballot(valid && bmx[g] >= target);
                if (m) bstar = c0 + __builtin_ctzll(m);
            }
            if (bstar >= 0 && valid && g > bstar) suf = fminf(suf, bmn[g]);
        }
        if (bstar < 0) return N;  // every cum < target
        suf = fminf(suf, __shfl_xor(suf, 1, 64));
        suf = fminf(suf, __shfl_xor(suf, 2, 64));
        suf = fminf(suf, __shfl_xor(suf, 4, 64));
        suf = fminf(suf, __shfl_xor(suf, 8, 64));
        suf = fminf(suf, __shfl_xor(suf, 16, 64));
        suf = fminf(suf, __shfl_xor(suf, 32, 64));
        if (suf >= target) {
            const int base = bstar << 6, c = min(64, N - base);
            const float v = lane < c ? d0[base + lane] : 0.0f;
            float run = bstar > 0 ? ck[bstar - 1] : 0.0f, mine = 0.0f;
            for (int l = 0; l < c; ++l) {
                run = fa(run, readlane_f(v, l));
                if (lane == l) mine = run;
            }
            const uint64_t ge = __ballot(lane < c && mine >= target);
            if (ge) {
                const int j = __builtin_ctzll(ge);
                if (__ballot(lane >= j && lane < c && !(mine >= target)) == 0ull) return base + j;
            }
        }
    }
    int first = 0, count = N;
    while (count > 0) {
        const int half = count >> 1;
        const int mid = first + half;
        if (target > cum_at(d0, ck, mid, lane)) {
            first = mid + 1;
            count -= half + 1;
        } else {
            count = half;
        }
    }
    return first;
}

}  // namespace

// dynamic LDS bytes of a frame with N points
__host__ __device__ constexpr size_t yakmo_dyn_lds(int N) { return size_t(3) * size_t((N + 63) / 64) * sizeof(float); }

// BIG: frames of more than kYMaxLds points (long -fl frames at small ChunkSize)
// keep the chosen-point bitmap and the per-block prefix summaries in HBM
// (gbits / gsum, frame slices at (n_off >> 5) + fi words and 3 ((n_off >> 6) +
// fi) floats) instead of LDS; one workgroup's own stores and loads, ordered by
// program order and the pick-end barrier (L1 is per CU and write-through)
template <int D, bool BIG>
__global__ __launch_bounds__(kYThreads) void yakmo_seed2_kernel(const ReduceFrame* __restrict__ frames, int nframes,
                                                                 const float* __restrict__ Xall, float* __restrict__ Call,
                                                                 float* __restrict__ f_scratch, int* __restrict__ i_scratch,
                                                                 float* __restrict__ gsum, uint32_t* __restrict__ gbits) {
    __shared__ YakmoShared sh;
    extern __shared__ __attribute__((aligned(16))) float ydyn[];
    const int fi = blockIdx.x;
    if (fi >= nframes) return;
    const ReduceFrame fr = frames[fi];
    const int N = fr.N, K = fr.K;
    const int nb = (N + 63) >> 6;
    float* const sum0 = BIG ? gsum + 3 * ((fr.n_off >> 6) + fi) : ydyn;
    float* ck = sum0;
    float* bmn = sum0 + nb;
    float* bmx = sum0 + 2 * nb;
    uint32_t* const chosen = BIG ? gbits + (fr.n_off >> 5) + fi : sh.chosen;
    const int nchosen = BIG ? (N + 31) >> 5 : kYBits;
    const float* __restrict__ X = Xall + fr.x_off;
    float* C = Call + fr.c_off;
    float* d0 = f_scratch + fr.n_off * 4;
    float* norm = d0 + N;
    int* order = reinterpret_cast<int*>(norm + N);  // N point indices (cluster order)
    uint16_t* id16 = reinterpret_cast<uint16_t*>(order + N);  // seed of each point (K <= 4096), the picks' copy
    int* idv = i_scratch + fr.n_off;  // seeding assignment
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    // yakmo point norm: norm += v*v (f32, in order) (@0x1800015cb)
    float xm = 0.0f;
    for (int n = tid; n < N; n += kYThreads) {
        const float* x = X + (int64_t)n * D;
        float s = 0.0f;
#pragma unroll
        for (int j = 0; j < D; ++j) s = fa(s, fm(x[j], x[j]));
        norm[n] = s;
        xm = fmaxf(xm, __builtin_isnan(s) ? 3.4028235e38f : s);
    }
    for (int w = tid; w < nchosen; w += kYThreads) chosen[w] = 0u;
    if (tid == 0) sh.xmax = 0.0f;
    __syncthreads();
    atomicMax(reinterpret_cast<unsigned*>(&sh.xmax), __float_as_uint(xm));  // non-negative floats order as integers
    __syncthreads();

    uint64_t rx = 123456789ull, ry = 362436069ull, rz = 521288629ull, rw = 88675123ull;
    float total = 0.0f;
    constexpr int kYPts = yakmo_pts<D>();
    constexpr int BLK = kYDist * kYPts;  // points per pipeline step
    const int nblk = (N + BLK - 1) / BLK;
    const bool idle = yakmo_idle_wave(wave);
    const int dt = (wave == 0 || idle) ? -1 : yakmo_dist_index(wave, lane);  // distance thread index
    YST_DECL
    for (int i = 0; i < K; ++i) {
        // ---- pick (wave 0; the RNG runs redundantly in every thread)
        const uint64_t t = rx ^ (rx << 11);
        rx = ry;
        ry = rz;
        rz = rw;
        rw = rw ^ (rw >> 19) ^ t ^ (t >> 8);
        const float r = (float)((double)rw * 5.42101086242752217e-20);  // f32(f64(w) * 2^-64)
        // distance waves: this pick's first seed ids / d0 are in flight during the pick
        float pd[kYPre][kYPts];
        int pa[kYPre][kYPts];
        if (dt >= 0) {
#pragma unroll
            for (int q = 0; q < kYPre; ++q)
#pragma unroll
                for (int p = 0; p < kYPts; ++p) {
                    int n = q * BLK + p * kYDist + dt;
                    asm volatile("" : "+v"(n));  // (no hoisted 64-bit address per slot)
                    pd[q][p] = 0.0f;
                    pa[q][p] = 0;
                    if (i > 0 && n < N) {
                        pd[q][p] = d0[n];
                        pa[q][p] = id16[n];
                    }
                }
        }
        if (wave == 0) {
            uint32_t idx;
            if (i == 0) {
                idx = (uint32_t)(int64_t)floorf(fm(r, (float)N));
            } else {
                idx = (uint32_t)(int64_t)(float)pick_lower_bound(fm(r, total), total, N, ck, bmn, bmx, d0, lane);
            }
            // collision walk (@0x180001b20) and clamp (@0x180001c50)
            while (idx < (uint32_t)N && ((chosen[idx >> 5] >> (idx & 31)) & 1u))
                idx = (idx < (uint32_t)(N - 1)) ? idx + 1 : 0u;
            if (idx >= (uint32_t)N) idx = (uint32_t)(N - 1);
            if (lane == 0) {
                chosen[idx >> 5] |= 1u << (idx & 31);
                const float cn = norm[idx];
                sh.cn = cn;
                sh.cmax = i == 0 ? cn : fmaxf(sh.cmax, cn);
            }
            if (lane < D) {
                const float v = X[(int64_t)idx * D + lane];
                sh.c[lane] = v;
                C[(int64_t)i * D + lane] = v;  // the seeds (C is overwritten by the means at the end)
            }
            YST(0)
        }
        lds_barrier();  // the seed (LDS); its C row is read from the next pick on
        const bool chain = i < K - 1;
        if (wave == 0) {
            YST(3)
            lds_barrier();  // the distance waves' seed-distance table
            YST(3)
            // sequential f32 prefix over the blocks as they complete (encoder's cum[], DLL @0x180001e74)
            float run = 0.0f;
            // back-off: after consecutive fast-path calls that accept nothing
            // (a total hovering around zero in quiet real audio changes binade
            // at nearly every point), the next 1, 3, 7, 15 blocks go point by
            // point without trying
            int fails = 0, skipfast = 0;
            for (int b = 0; b <= nblk; ++b) {
                if (chain && b > 0) {
                    const int base = (b - 1) * BLK;
                    const float* rg = sh.ring[(b - 1) & 1];
                    const int cnt = min(BLK, N - base);
                    int s = 0;
                    while (s < cnt) {
                        const int full = (cnt - s) >> 6;
                        if (full > 0 && skipfast == 0) {
                            // (at most 8 blocks left, e.g. after a break: 8 points per lane)
                            int k;
                            if (BLK / 64 == 16 && full <= 8)
                                k = chain_fast<8>(rg, s, full, lane, &run, ck, bmn, bmx, (base + s) >> 6);
                            else
                                k = chain_fast<BLK / 64>(rg, s, full, lane, &run, ck, bmn, bmx, (base + s) >> 6);
                            s += k << 6;
                            fails = k > 0 ? 0 : min(fails + 1, 5);
                            skipfast = (1 << fails) >> 1;
                            skipfast = skipfast > 0 ? skipfast - 1 : 0;
                            YST(1) YCNT(4)
                            if (s >= cnt) break;
                        } else if (skipfast > 0) {
                            --skipfast;
                        }
                        // the block at s breaks a fast-path condition (or is the last, partial one)
                        const int c = min(64, cnt - s);
                        chain_seq(rg, s, c, lane, &run, ck, bmn, bmx, (base + s) >> 6);
                        s += c;
                        YST(2) YCNT(5)
                    }
                }
                step_barrier(b == nblk);
                YST(3)
            }
            total = run;
        } else if (idle) {
            lds_barrier();
            for (int b = 0; b <= nblk; ++b) step_barrier(b == nblk);
        } else {
            float c[D];
#pragma unroll
            for (int j = 0; j < D; ++j) c[j] = sh.c[j];
            const float cn = sh.cn;
            const float cmax = sh.cmax, xmax = sh.xmax;
            // Seed-distance table: sdlo[a] <= |c_i - c_a|^2 (the f32 sum of squared
            // differences, lowered by 2^-16 relative to cover its rounding).
#pragma unroll 4  // (up to four rows' loads in flight before their sums)
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
            lds_barrier();
            YST(8)
            // Elkan skip: with E = (max|x|^2 + cmax) 2^-16 >= the rounding error of any of
            // the DLL's expanded-form distances from x (< 80 u (|x|^2 + |c|^2)), the
            // computed d0 = d(x, c_a) and d(x, c_i) are within E of the true squares, so
            // |c_i - c_a| >= 2 sqrt(max(d0, 0) + E) implies d(x, c_i) >= d0: no strict
            // improvement, and the point's X row need not be read for this pick.
            const float e = fm(fa(xmax, cmax), 1.52587891e-05f);
            auto skip_of = [&](float dold, int a) -> bool {
                if (i == 0) return false;
                const float need = fm(fm(fa(fmaxf(dold, 0.0f), e), 4.0f), 1.00000381f);
                return sh.sdlo[a] >= need;
            };
            // pipeline: step b computes block b (kYPts points per thread, kYDist
            // apart); the X rows of block b + XD (when not skipped) and the d0 /
            // seed ids of block b + kYPre are loaded meanwhile
            constexpr int XD = kYXD;  // X-row look-ahead in steps (a step is 1024 points)
            float xv[XD][kYPts][D];
            float xnv[XD][kYPts];  // yakmo's |x|^2 (norm[], computed at the start)
            bool skip[XD][kYPts];
#pragma unroll
            for (int q = 0; q < XD; ++q)
#pragma unroll
                for (int p = 0; p < kYPts; ++p) {
                    const int n = q * BLK + p * kYDist + dt;
                    skip[q][p] = true;
                    if (n < N) {
                        skip[q][p] = skip_of(pd[q][p], pa[q][p]);
                        if (!skip[q][p]) {
                            xnv[q][p] = norm[n];
#pragma unroll
                            for (int j = 0; j < D; ++j) xv[q][p][j] = X[(int64_t)n * D + j];
                        }
                    }
                }
            for (int b0 = 0; b0 <= nblk; b0 += kYPre) {
#pragma unroll
                for (int u = 0; u < kYPre; ++u) {
                    const int b = b0 + u;
                    if (b > nblk) break;
                    const int s2 = u % XD;
#pragma unroll
                    for (int p = 0; p < kYPts; ++p) {
                        const int n = b * BLK + p * kYDist + dt;
                        if (b < nblk && n < N) {
                            float dn = pd[u][p];
                            if (!skip[s2][p]) {
                                float d = fa(fa(cn, xnv[s2][p]), 0.0f);
#pragma unroll
                                for (int j = 0; j < D; ++j) d = fs(d, fm(fa(xv[s2][p][j], xv[s2][p][j]), c[j]));
                                if (i == 0 || dn > d) {
                                    dn = d;
                                    d0[n] = d;
                                    idv[n] = i;
                                    id16[n] = (uint16_t)i;
                                }
                            }
                            sh.ring[b & 1][p * kYDist + dt] = dn;
                        }
                    }
#pragma unroll
                    for (int p = 0; p < kYPts; ++p) {
                        const int n = b * BLK + p * kYDist + dt;
                        // block b + XD: skip decision and X rows (slot s2 is free now)
                        const int n2 = n + XD * BLK;
                        skip[s2][p] = true;
                        if (b + XD < nblk && n2 < N) {
                            skip[s2][p] = skip_of(pd[(u + XD) % kYPre][p], pa[(u + XD) % kYPre][p]);
                            if (!skip[s2][p]) {
                                xnv[s2][p] = norm[n2];
#pragma unroll
                                for (int j = 0; j < D; ++j) xv[s2][p][j] = X[(int64_t)n2 * D + j];
                            }
                        }
                        // block b + kYPre: d0 and seed id (slot u is free now)
                        const int n4 = n + kYPre * BLK;
                        if (i > 0 && b + kYPre < nblk && n4 < N) {
                            pd[u][p] = d0[n4];
                            pa[u][p] = id16[n4];
                        }
                    }
                    YST(9)
                    step_barrier(b == nblk);
                    YST(10)
                }
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

// Test hook (tests/test_gpu_yakmo_chain.py): one wave runs chain_fast<PPL> on
// a ring of nbk 64-point blocks starting at run, so that the integer prefix
// path (ties, negative runs, zero runs, NaN / inf, binade crossings) is
// checked point for point against the sequential f32 chain it replaces.
template <int PPL>
__global__ __launch_bounds__(64) void yakmo_chain_test_kernel(const float* __restrict__ pts, int nbk, float run,
                                                              int* __restrict__ k_out, float* __restrict__ out) {
    __shared__ alignas(16) float ring[64 * PPL];
    __shared__ float ck[64], bmn[64], bmx[64];
    const int lane = threadIdx.x;
    for (int i = lane; i < 64 * PPL; i += 64) ring[i] = i < 64 * nbk ? pts[i] : 0.0f;
    for (int i = lane; i < 64; i += 64) ck[i] = bmn[i] = bmx[i] = __builtin_nanf("");
    __syncthreads();
    float r = run;
    const int k = chain_fast<PPL>(ring, 0, nbk, lane, &r, ck, bmn, bmx, 0);
    __syncthreads();
    if (lane == 0) {
        *k_out = k;
        out[0] = r;
    }
    if (lane < nbk) {
        out[1 + lane] = ck[lane];
        out[1 + 64 + lane] = bmn[lane];
        out[1 + 128 + lane] = bmx[lane];
    }
}

}  // namespace gsc

using namespace gsc;

// nbk <= 64 / (64 / PPL) blocks: out = run, then ck[64], bmn[64], bmx[64]
extern "C" hipError_t gsc_launch_yakmo_chain_test(int ppl, const float* pts, int nbk, float run, int* k_out,
                                                  float* out) {
    if (nbk < 1 || nbk > ppl || (ppl != 8 && ppl != 16)) return hipErrorInvalidValue;
    if (ppl == 8)
        hipLaunchKernelGGL(yakmo_chain_test_kernel<8>, dim3(1), dim3(64), 0, nullptr, pts, nbk, run, k_out, out);
    else
        hipLaunchKernelGGL(yakmo_chain_test_kernel<16>, dim3(1), dim3(64), 0, nullptr, pts, nbk, run, k_out, out);
    return hipGetLastError();
}

// gsum / gbits: HBM state of frames over kYMaxLds points (see yakmo_seed2_kernel;
// gsc_yakmo_big_floats / _words give the sizes); unused otherwise
extern "C" hipError_t gsc_launch_yakmo(int D, const ReduceFrame* frames, int nframes, const float* X, float* C,
                                       float* fs, int* is, float* gsum, uint32_t* gbits, int max_n, hipStream_t st) {
    dim3 grid(nframes), block(kYThreads);
    const bool big = max_n > kYMaxLds;
    if (big && (!gsum || !gbits)) return hipErrorInvalidValue;
    const size_t shm = big ? 0 : yakmo_dyn_lds(max_n);
    hipError_t e = hipSuccess;
    switch (D) {
#define YK(DV, B)                                                                                                 \
    e = hipFuncSetAttribute((const void*)yakmo_seed2_kernel<DV, B>, hipFuncAttributeMaxDynamicSharedMemorySize,    \
                            (int)shm);                                                                            \
    if (e != hipSuccess) return e;                                                                                \
    hipLaunchKernelGGL((yakmo_seed2_kernel<DV, B>), grid, block, shm, st, frames, nframes, X, C, fs, is, gsum, gbits);
    case 8:
        if (big) { YK(8, true) } else { YK(8, false) }
        break;
    case 16:
        if (big) { YK(16, true) } else { YK(16, false) }
        break;
    case 32:
        if (big) { YK(32, true) } else { YK(32, false) }
        break;
#undef YK
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// HBM state of frames over kYMaxLds points: prefix summaries (floats) and chosen bitmaps (words)
// for nframes frames of total_points points
extern "C" size_t gsc_yakmo_big_floats(int64_t total_points, int nframes) {
    return size_t(3) * size_t(total_points / 64 + nframes + 1);
}
extern "C" size_t gsc_yakmo_big_words(int64_t total_points, int nframes) { return size_t(total_points / 32 + nframes + 1); }
extern "C" int gsc_yakmo_max_lds_points(void) { return kYMaxLds; }
