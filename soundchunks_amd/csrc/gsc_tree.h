// Shared device code of the KNNScanReduce kernels (gsc_kernels.hip: generic
// per-search kernel; gsc_scan.hip: batched speculative kernel).
//
//   KdTree          ANN_KD_STD kd-tree (bs = 1) over the centroids of one
//                   pass, in LDS, heap-indexed (root 0, children 2h+1 / 2h+2).
//   build_tree      annMaxSpread + annMedianSplit level by level
//                   (ANN.dll @0x180015260, @0x180015680).
//   scan_exact_dfs  ANN's k = 1 standard search (annkSearch @0x1800124b0)
//                   over precomputed live leaf distances (stale tree).
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "gsc_device.h"

namespace gsc {

__device__ __forceinline__ float fadd(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fsub(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ float fmul(float a, float b) { return __fmul_rn(a, b); }

__device__ __forceinline__ int lane_id() { return __lane_id(); }

template <typename T>
__device__ __forceinline__ T ld_relaxed(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct KdTree {
    float cv[kMaxInternal + 1];    // cut value per split node
    float lo[kMaxInternal + 1];    // cd_bnds lo / hi of the split node's cell
    float hi[kMaxInternal + 1];
    uint16_t pidx[kMaxK];          // kd-leaf position -> centroid id
    uint8_t cd[kMaxInternal + 1];  // cut dimension
    float bnd_lo[32], bnd_hi[32];  // annEnclRect of the pass's centroids
};

// ---------------------------------------------------------------------------
// Parallel build for K = 2^LOGK (the batched scan kernel).  ANN's build is
// order dependent only through ties: annMaxSpread's min/max, the median's
// left set (the n_lo smallest cut values) and the cut value (max of the left
// set + min of the right set) / 2 are functions of each node's point SET as
// long as the two values at the median boundary differ.  Then the children's
// sets, and by induction the whole tree and its leaf order, do not depend on
// the order quickselect leaves inside a segment.  So each level: per-node
// spreads by reductions, cut values gathered, every segment bitonic-sorted in
// LDS, the left half taken.  A node whose boundary values tie (or compare
// unordered) makes the function return false: the caller then runs the
// sequential build_tree, which reproduces quickselect's tie order exactly.
//   val: K floats of LDS scratch; red: 2*D*(K/512) floats of LDS scratch.
// ---------------------------------------------------------------------------
template <int D, int LOGK, int NT>
__device__ bool build_tree_fast(KdTree& t, float* __restrict__ val, float* __restrict__ red,
                                const float* __restrict__ C, int* tie) {
    constexpr int K = 1 << LOGK;
    constexpr int PT = K / NT;  // kd-leaf positions per thread
    static_assert(PT * NT == K && (PT == 4 || PT == 8), "positions per thread");
    const int tid = threadIdx.x, wave = tid >> 6;
    const int p0 = tid * PT;
    for (int p = tid; p < K; p += NT) t.pidx[p] = (uint16_t)p;
    if (tid == 0) *tie = 0;
    __syncthreads();
    for (int L = 0; L < LOGK; ++L) {
        const int S = K >> L;  // segment (node) size at this level
        const int first = (1 << L) - 1;
        // ---- annMaxSpread per node: min / max per dimension -> cut dimension
        if (S >= PT) {
            float mn[D], mx[D];
            {
                const float* r = C + (int64_t)t.pidx[p0] * D;
#pragma unroll
                for (int d = 0; d < D; ++d) mn[d] = mx[d] = r[d];
            }
#pragma unroll
            for (int i = 1; i < PT; ++i) {
                const float* r = C + (int64_t)t.pidx[p0 + i] * D;
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const float c = r[d];
                    mn[d] = fminf(mn[d], c);
                    mx[d] = fmaxf(mx[d], c);
                }
            }
            const int G = S / PT;  // threads per node
            const int GW = G < 64 ? G : 64;
            for (int o = 1; o < GW; o <<= 1) {
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    mn[d] = fminf(mn[d], __shfl_xor(mn[d], o));
                    mx[d] = fmaxf(mx[d], __shfl_xor(mx[d], o));
                }
            }
            if (G > 64) {  // node spans G/64 waves
                if ((tid & 63) == 0) {
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        red[wave * 2 * D + d] = mn[d];
                        red[wave * 2 * D + D + d] = mx[d];
                    }
                }
                __syncthreads();
                const int wn = G / 64, w0 = (wave / wn) * wn;
                for (int w = w0; w < w0 + wn; ++w) {
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        mn[d] = fminf(mn[d], red[w * 2 * D + d]);
                        mx[d] = fmaxf(mx[d], red[w * 2 * D + D + d]);
                    }
                }
            }
            if (p0 % S == 0) {
                int cdim = 0;
                float max_spr = 0.0f;
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const float spr = fsub(mx[d], mn[d]);
                    if (spr > max_spr) {
                        max_spr = spr;
                        cdim = d;
                    }
                }
                t.cd[first + p0 / S] = (uint8_t)cdim;
                if (L == 0) {  // annEnclRect of all centroids
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        t.bnd_lo[d] = mn[d];
                        t.bnd_hi[d] = mx[d];
                    }
                }
            }
        } else {  // several nodes per thread
            for (int g = 0; g < PT / S; ++g) {
                float mn[D], mx[D];
                const int pb = p0 + g * S;
                {
                    const float* r = C + (int64_t)t.pidx[pb] * D;
#pragma unroll
                    for (int d = 0; d < D; ++d) mn[d] = mx[d] = r[d];
                }
                for (int i = 1; i < S; ++i) {
                    const float* r = C + (int64_t)t.pidx[pb + i] * D;
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        const float c = r[d];
                        mn[d] = fminf(mn[d], c);
                        mx[d] = fmaxf(mx[d], c);
                    }
                }
                int cdim = 0;
                float max_spr = 0.0f;
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const float spr = fsub(mx[d], mn[d]);
                    if (spr > max_spr) {
                        max_spr = spr;
                        cdim = d;
                    }
                }
                t.cd[first + pb / S] = (uint8_t)cdim;
            }
        }
        __syncthreads();
        // ---- cut-dimension values of every position
#pragma unroll
        for (int i = 0; i < PT; ++i) {
            const int p = p0 + i;
            val[p] = C[(int64_t)t.pidx[p] * D + t.cd[first + p / S]];
        }
        __syncthreads();
        // ---- bitonic sort of every segment (ascending; order among equal values is free)
        for (int k = 2; k <= S; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
                for (int e = 0; e < PT / 2; ++e) {
                    const int i = tid + e * NT;
                    const int a = ((i & ~(j - 1)) << 1) | (i & (j - 1));
                    const int b = a + j;
                    const bool up = k == S || (a & k) == 0;
                    const float va = val[a], vb = val[b];
                    if (up ? (va > vb) : (va < vb)) {
                        val[a] = vb;
                        val[b] = va;
                        const uint16_t ia = t.pidx[a];
                        t.pidx[a] = t.pidx[b];
                        t.pidx[b] = ia;
                    }
                }
                __syncthreads();
            }
        }
        // ---- per node: cut value, tie check, cell bounds on the cut dimension
        for (int node = tid; node < (1 << L); node += NT) {
            const int h = first + node, s = node * S, nl = S >> 1;
            const float a = val[s + nl - 1], b = val[s + nl];
            if (!(a < b)) *tie = 1;
            const int cdim = t.cd[h];
            float lov = t.bnd_lo[cdim], hiv = t.bnd_hi[cdim];
            int an = 0;
            const int path = h + 1;
            for (int bl = L - 1; bl >= 0; --bl) {
                const int right = (path >> bl) & 1;
                if (t.cd[an] == cdim) {
                    if (right) lov = t.cv[an];
                    else hiv = t.cv[an];
                }
                an = 2 * an + 1 + right;
            }
            t.cv[h] = (float)((double)fadd(a, b) / 2.0);
            t.lo[h] = lov;
            t.hi[h] = hiv;
        }
        __syncthreads();
    }
    return *tie == 0;
}

// annMedianSplit (ANN.dll @0x180015680) on one node's segment, one thread:
// quickselect of the n_lo = n/2 smallest cut-dimension values (pidx and their
// staged values val move together; NaN values compare false everywhere, as in
// the DLL), then the largest of the low side moved to n_lo - 1
__device__ __forceinline__ void median_split(uint16_t* __restrict__ pidx, float* __restrict__ val, int n) {
    const int n_lo = n >> 1;
    int l = 0, r = n - 1;
#define PSWAP(a, b)                 \
    {                               \
        const uint16_t t_ = pidx[a]; \
        pidx[a] = pidx[b];          \
        pidx[b] = t_;               \
        const float v_ = val[a];    \
        val[a] = val[b];            \
        val[b] = v_;                \
    }
    while (l < r) {
        int i = (r + l) / 2;
        int k;
        if (val[i] > val[r]) PSWAP(i, r)
        PSWAP(l, i);
        const float c = val[l];
        i = l;
        k = r;
        for (;;) {
            while (val[++i] < c) {}
            while (val[--k] > c) {}
            if (i < k) PSWAP(i, k) else break;
        }
        PSWAP(l, k);
        if (k > n_lo) r = k - 1;
        else if (k < n_lo) l = k + 1;
        else break;
    }
    if (n_lo > 0) {
        float c = val[0];
        int k = 0;
        for (int i = 1; i < n_lo; ++i)
            if (val[i] > c) {
                c = val[i];
                k = i;
            }
        PSWAP(n_lo - 1, k);
    }
#undef PSWAP
}

// ---------------------------------------------------------------------------
// Exact build for K = 2^LOGK centroids some of which are NaN (yakmo's 0/0
// means): quickselect's order matters there (NaN compares false), so each
// node's median split runs sequentially on one thread (median_split, as in
// build_tree) -- but on cut values staged in LDS by all threads, and with the
// node spreads computed by all threads.  annMaxSpread's sequential min / max
// start at the segment's first point and never take a NaN, so per dimension
// the spread is NaN (never the cut dimension) when the first point's value is
// NaN, else max - min over the non-NaN values (fminf / fmaxf skip NaN); the
// enclosing rectangle likewise starts at point 0.
//   val: K floats of LDS scratch; red: 2*D*(K/512) floats of LDS scratch.
// ---------------------------------------------------------------------------
template <int D, int LOGK, int NT>
__device__ void build_tree_nan(KdTree& t, float* __restrict__ val, float* __restrict__ red,
                               const float* __restrict__ C) {
    constexpr int K = 1 << LOGK;
    constexpr int PT = K / NT;  // kd-leaf positions per thread
    static_assert(PT * NT == K && (PT == 4 || PT == 8), "positions per thread");
    const int tid = threadIdx.x, wave = tid >> 6;
    const int p0 = tid * PT;
    for (int p = tid; p < K; p += NT) t.pidx[p] = (uint16_t)p;
    __syncthreads();
    // cut dimension of the node whose segment starts at position sb, from its min / max
    auto pick = [&](int sb, const float (&mn)[D], const float (&mx)[D]) {
        const float* f = C + (int64_t)t.pidx[sb] * D;  // the segment's first point
        int cdim = 0;
        float max_spr = 0.0f;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const float spr = f[d] != f[d] ? f[d] : fsub(mx[d], mn[d]);
            if (spr > max_spr) {
                max_spr = spr;
                cdim = d;
            }
        }
        return cdim;
    };
    for (int L = 0; L < LOGK; ++L) {
        const int S = K >> L;
        const int first = (1 << L) - 1;
        if (S >= PT) {
            float mn[D], mx[D];
#pragma unroll
            for (int d = 0; d < D; ++d) {
                mn[d] = __builtin_nanf("");
                mx[d] = __builtin_nanf("");
            }
#pragma unroll
            for (int i = 0; i < PT; ++i) {
                const float* r = C + (int64_t)t.pidx[p0 + i] * D;
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    mn[d] = fminf(mn[d], r[d]);
                    mx[d] = fmaxf(mx[d], r[d]);
                }
            }
            const int G = S / PT;
            const int GW = G < 64 ? G : 64;
            for (int o = 1; o < GW; o <<= 1) {
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    mn[d] = fminf(mn[d], __shfl_xor(mn[d], o));
                    mx[d] = fmaxf(mx[d], __shfl_xor(mx[d], o));
                }
            }
            if (G > 64) {
                if ((tid & 63) == 0) {
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        red[wave * 2 * D + d] = mn[d];
                        red[wave * 2 * D + D + d] = mx[d];
                    }
                }
                __syncthreads();
                const int wn = G / 64, w0 = (wave / wn) * wn;
                for (int w = w0; w < w0 + wn; ++w) {
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        mn[d] = fminf(mn[d], red[w * 2 * D + d]);
                        mx[d] = fmaxf(mx[d], red[w * 2 * D + D + d]);
                    }
                }
            }
            if (p0 % S == 0) {
                t.cd[first + p0 / S] = (uint8_t)pick(p0, mn, mx);
                if (L == 0) {  // annEnclRect from point 0
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        const float c0 = C[d];
                        t.bnd_lo[d] = c0 != c0 ? c0 : mn[d];
                        t.bnd_hi[d] = c0 != c0 ? c0 : mx[d];
                    }
                }
            }
        } else {
            for (int g = 0; g < PT / S; ++g) {
                float mn[D], mx[D];
                const int pb = p0 + g * S;
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    mn[d] = __builtin_nanf("");
                    mx[d] = __builtin_nanf("");
                }
                for (int i = 0; i < S; ++i) {
                    const float* r = C + (int64_t)t.pidx[pb + i] * D;
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        mn[d] = fminf(mn[d], r[d]);
                        mx[d] = fmaxf(mx[d], r[d]);
                    }
                }
                t.cd[first + pb / S] = (uint8_t)pick(pb, mn, mx);
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PT; ++i) {  // cut-dimension values, staged in LDS
            const int p = p0 + i;
            val[p] = C[(int64_t)t.pidx[p] * D + t.cd[first + p / S]];
        }
        __syncthreads();
        for (int node = tid; node < (1 << L); node += NT) {  // quickselect, one thread per node
            const int h = first + node, sb = node * S, nl = S >> 1;
            median_split(t.pidx + sb, val + sb, S);
            const int cdim = t.cd[h];
            float lov = t.bnd_lo[cdim], hiv = t.bnd_hi[cdim];
            int a = 0;
            const int path = h + 1;
            for (int bl = L - 1; bl >= 0; --bl) {
                const int right = (path >> bl) & 1;
                if (t.cd[a] == cdim) {
                    if (right) lov = t.cv[a];
                    else hiv = t.cv[a];
                }
                a = 2 * a + 1 + right;
            }
            t.cv[h] = (float)((double)fadd(val[sb + nl - 1], val[sb + nl]) / 2.0);
            t.lo[h] = lov;
            t.hi[h] = hiv;
        }
        __syncthreads();
    }
}

// segment of heap node h (root 0, children 2h+1 / 2h+2, n_lo = n/2)
__device__ __forceinline__ void node_segment(int h, int K, int& s, int& n, int& depth) {
    s = 0;
    n = K;
    depth = 0;
    int path = h + 1;
    int lvl = 31 - __clz(path);
    depth = lvl;
    for (int l = lvl - 1; l >= 0; --l) {
        const int half = n >> 1;
        if ((path >> l) & 1) {
            s += half;
            n -= half;
        } else {
            n = half;
        }
    }
}

// Embeds ANN's tree over kr points (build_tree: heap-indexed, n_lo = n/2,
// compact leaf positions 0..kr-1) into the complete tree of 2^LOGK leaves the
// batched kernel lays out in registers: node h keeps its heap index (the same
// root path); a point's leaf position is its root path over LOGK levels,
// continuing below its own leaf the way node_segment does (a node of one
// point hands it to its high child).  Those nodes below a point (n <= 1)
// become pass-through splits that send every query to the high child
// (cut value -inf, cell [-inf, inf]): ANN's search and the padded one reach
// the real leaves in the same order under the same conditions, and the
// padding leaves (pidx 0xFFFF) carry +inf distances, so they are never a
// result and never an improvement.  stage: kr ints of scratch.
template <int LOGK>
__device__ void pad_tree(KdTree& t, int* __restrict__ stage, int kr, int tid, int nt) {
    constexpr int K = 1 << LOGK;
    __syncthreads();  // build_tree is done with the scratch
    for (int i = tid; i < kr; i += nt) stage[i] = t.pidx[i];
    __syncthreads();
    for (int p = tid; p < K; p += nt) t.pidx[p] = 0xFFFF;
    __syncthreads();
    for (int i = tid; i < kr; i += nt) {
        int s = 0, n = kr, pos = 0;
        for (int l = 0; l < LOGK; ++l) {
            const int half = n >> 1;
            const int hi = i >= s + half ? 1 : 0;
            if (hi) {
                s += half;
                n -= half;
            } else {
                n = half;
            }
            pos = (pos << 1) | hi;
        }
        t.pidx[pos] = (uint16_t)stage[i];
    }
    for (int h = tid; h < K - 1; h += nt) {
        int s, n, depth;
        node_segment(h, kr, s, n, depth);
        if (n <= 1) {
            t.cd[h] = 0;
            t.cv[h] = -__builtin_inff();
            t.lo[h] = -__builtin_inff();
            t.hi[h] = __builtin_inff();
        }
    }
    __syncthreads();
}

template <int D>
__device__ void build_tree(KdTree& sh, float* __restrict__ scratch, const float* __restrict__ C, int K) {
    const int tid = threadIdx.x;
    const int nthr = blockDim.x;
    for (int p = tid; p < K; p += nthr) sh.pidx[p] = (uint16_t)p;
    // annEnclRect: sequential min/max from PA(0,d); NaNs never win a compare
    if (tid < D) {
        const int d = tid;
        float lo = C[d], hi = C[d];
        for (int i = 0; i < K; ++i) {
            const float v = C[(int64_t)i * D + d];
            if (v < lo) lo = v;
            else if (v > hi) hi = v;
        }
        sh.bnd_lo[d] = lo;
        sh.bnd_hi[d] = hi;
    }
    __syncthreads();
    // split level by level; one thread per node runs ANN's exact sequential code
    for (int level = 0; level < 12; ++level) {
        const int first = (1 << level) - 1;
        const int count = 1 << level;
        for (int j = tid; j < count; j += nthr) {
            const int h = first + j;
            if (h > kMaxInternal - 1) continue;
            int s, n, depth;
            node_segment(h, K, s, n, depth);
            if (n < 2) continue;
            uint16_t* pidx = sh.pidx + s;
            // annMaxSpread: first dim with strictly largest spread
            int cdim = 0;
            float max_spr = 0.0f;
            {
                float mn[D], mx[D];
                const float* p0 = C + (int64_t)pidx[0] * D;
#pragma unroll
                for (int d = 0; d < D; ++d) mn[d] = mx[d] = p0[d];
                for (int i = 1; i < n; ++i) {
                    const float* pp = C + (int64_t)pidx[i] * D;
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        const float c = pp[d];
                        if (c < mn[d]) mn[d] = c;
                        else if (c > mx[d]) mx[d] = c;
                    }
                }
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const float spr = fsub(mx[d], mn[d]);
                    if (spr > max_spr) {
                        max_spr = spr;
                        cdim = d;
                    }
                }
            }
            float* val = scratch + s;  // cut-dim values of the segment
            for (int i = 0; i < n; ++i) val[i] = C[(int64_t)pidx[i] * D + cdim];
            const int n_lo = n >> 1;
            median_split(pidx, val, n);
            const float cvv = (float)((double)fadd(val[n_lo - 1], val[n_lo]) / 2.0);
            // node bounds: root rect narrowed by ancestors cutting the same dim
            float lov = sh.bnd_lo[cdim], hiv = sh.bnd_hi[cdim];
            {
                int a = 0;
                const int path = h + 1;
                for (int bl = depth - 1; bl >= 0; --bl) {
                    const int right = (path >> bl) & 1;
                    if (sh.cd[a] == cdim) {
                        if (right) lov = sh.cv[a];
                        else hiv = sh.cv[a];
                    }
                    a = 2 * a + 1 + right;
                }
            }
            sh.cd[h] = (uint8_t)cdim;
            sh.cv[h] = cvv;
            sh.lo[h] = lov;
            sh.hi[h] = hiv;
        }
        __syncthreads();
    }
}

// depth of the lowest common ancestor of kd-leaf positions p and q (p != q)
__device__ __forceinline__ int lca_depth(int p, int q, int K, int log2K, bool pow2) {
    if (pow2) return __clz(p ^ q) - (32 - log2K);
    int s = 0, n = K, depth = 0;
    for (;;) {
        const int half = n >> 1;
        const bool a = p >= s + half, b = q >= s + half;
        if (a != b) return depth;
        if (a) {
            s += half;
            n -= half;
        } else {
            n = half;
        }
        ++depth;
    }
}

// Exact ANN ann_search (k = 1, eps = 0) over the stale tree with the live
// distances already in dist[].  Single lane.  For a NaN leaf visited while
// the result list is still empty, ANN's early exit depends on the partial sum
// before the first NaN term; that is recomputed from the live mirror in C.
template <int D>
__device__ __noinline__ void scan_exact_dfs(const KdTree& sh, const float* __restrict__ dist, const float (&q)[D], int K,
                                            const float* __restrict__ C, int& out_pos, float& out_key) {
    int st_h[16], st_s[16], st_n[16];
    float st_box[16];
    int sp = 0, nmk = 0, best = -1;
    float key = FLT_MAX;
    float cur_box = 0.0f;
    for (int d = 0; d < D; ++d) {
        if (q[d] < sh.bnd_lo[d]) {
            const float t = fsub(sh.bnd_lo[d], q[d]);
            cur_box = fadd(cur_box, fmul(t, t));
        } else if (q[d] > sh.bnd_hi[d]) {
            const float t = fsub(q[d], sh.bnd_hi[d]);
            cur_box = fadd(cur_box, fmul(t, t));
        }
    }
    int h = 0, s = 0, n = K;
    for (;;) {
        if (n == 1) {
            // ANNkd_leaf::ann_search: skipped iff some partial sum exceeds min_dist
            const float dd = dist[s];
            const float min_dist = nmk == 1 ? key : FLT_MAX;
            float chk = dd;
            if (dd != dd) {
                const float* c = C + (int64_t)sh.pidx[s] * D;
                float pr = 0.0f;
                for (int d = 0; d < D; ++d) {
                    const float t = fsub(q[d], c[d]);
                    const float sq = fmul(t, t);
                    if (sq != sq) break;
                    pr = fadd(pr, sq);
                }
                chk = pr;
            }
            if (!(chk > min_dist)) {
                if (nmk == 0) {
                    key = dd;
                    best = s;
                    nmk = 1;
                } else if (key > dd) {
                    key = dd;
                    best = s;
                }
            }
            // return up the recursion: far child visited iff box' < max_key
            bool found = false;
            while (sp > 0) {
                --sp;
                const float mk = nmk == 1 ? key : FLT_MAX;
                if ((double)st_box[sp] < (double)mk) {
                    h = st_h[sp];
                    s = st_s[sp];
                    n = st_n[sp];
                    cur_box = st_box[sp];
                    found = true;
                    break;
                }
            }
            if (!found) break;
            continue;
        }
        // ANNkd_split::ann_search: descend near child, remember far child + box'
        const int half = n >> 1;
        const int cdim = sh.cd[h];
        const float qc = q[cdim];
        const float cut = fsub(qc, sh.cv[h]);
        float bd;
        int nh, ns, nn;
        if (cut < 0.0f) {
            bd = fsub(sh.lo[h], qc);
            nh = 2 * h + 1;
            ns = s;
            nn = half;
            st_h[sp] = 2 * h + 2;
            st_s[sp] = s + half;
            st_n[sp] = n - half;
        } else {
            bd = fsub(qc, sh.hi[h]);
            nh = 2 * h + 2;
            ns = s + half;
            nn = n - half;
            st_h[sp] = 2 * h + 1;
            st_s[sp] = s;
            st_n[sp] = half;
        }
        if (bd < 0.0f) bd = 0.0f;
        st_box[sp] = fadd(cur_box, fsub(fmul(cut, cut), fmul(bd, bd)));
        ++sp;
        h = nh;
        s = ns;
        n = nn;
    }
    out_pos = best;
    out_key = key;
}

template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (T*)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int uniform_int(int v) { return __builtin_amdgcn_readfirstlane(v); }
// a wave-uniform 64-bit offset (SGPRs).  Offset a kernel-argument pointer with
// it instead of passing the sum through uniform_ptr: the integer round trip of
// uniform_ptr hides the global address space, the compiler then emits FLAT
// loads / stores, and every FLAT op also counts in lgkmcnt -- the next LDS wait
// would wait for the HBM access too
__device__ __forceinline__ int64_t uniform_i64(int64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

}  // namespace gsc
