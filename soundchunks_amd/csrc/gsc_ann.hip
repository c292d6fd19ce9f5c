// GPU implementation of the ANN.dll surface bound by extern.pas:118-123
// (ann_kdtree_create / _search / _pri_search / _search_multi /
// _pri_search_multi).  The encoder itself uses the batched kernels in
// gsc_kernels.hip; this file serves the per-query drop-in ABI, so it favours
// exactness over speed: one workgroup builds the tree level by level with
// ANN 1.1's own split code per node (ANN.dll @0x180014620 ctor); a search computes every live point distance with all
// lanes of one workgroup and then walks ANN's DFS (@0x1800124b0 annkSearch)
// or best-bin-first search (@0x180011da0 annkPriSearch) on one lane.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "gsc_device.h"

namespace gsc {
namespace ann {

using Tree = gsc::AnnTree;

__device__ __forceinline__ float fa(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fs(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ float fm(float a, float b) { return __fmul_rn(a, b); }

// ---------------------------------------------------------------------------
// ANNkd_tree ctor with ANN_KD_STD, bs = 1 (ANN.dll @0x180014620): annEnclRect,
// then rkd_tree with kd_split = annMaxSpread + annMedianSplit (@0x180015260,
// @0x180015680), built level by level by one workgroup.  The nodes of a level
// own disjoint segments of pidx, so they split independently; within a node
// the reference's sequential quickselect runs unchanged on one lane (its
// swap order decides the leaf order among tied values, which the KNNFit
// overflow replay depends on), over the segment's cut values staged in a
// contiguous scratch array instead of the pidx -> pts gathers.  annMaxSpread
// is a min / max per dimension: "if (c < mn) mn = c; else if (c > mx) mx = c"
// from the segment's first point equals the NaN-ignoring min / max, except
// that a NaN first value stays NaN -- so long segments (>= kWaveSeg) reduce
// it over a wave's lanes.  Short ones run one node per lane.
// ---------------------------------------------------------------------------
constexpr int kBuildThreads = 256;
constexpr int kWaveSeg = 512;

// annMedianSplit on (pidx, val) of one segment; returns the cut value
__device__ float median_split_v(int* __restrict__ pidx, float* __restrict__ val, int n, int n_lo) {
    int l = 0, r = n - 1;
#define SWP(a, b)                   \
    {                               \
        const int x_ = pidx[a];     \
        pidx[a] = pidx[b];          \
        pidx[b] = x_;               \
        const float v_ = val[a];    \
        val[a] = val[b];            \
        val[b] = v_;                \
    }
    while (l < r) {
        int i = (r + l) / 2, k;
        if (val[i] > val[r]) SWP(i, r)
        SWP(l, i);
        const float c = val[l];
        i = l;
        k = r;
        for (;;) {
            while (val[++i] < c) {}
            while (val[--k] > c) {}
            if (i < k) SWP(i, k) else break;
        }
        SWP(l, k);
        if (k > n_lo) r = k - 1;
        else if (k < n_lo) l = k + 1;
        else break;
    }
    if (n_lo > 0) {
        float c = val[0];
        int k = 0;
        for (int i = 1; i < n_lo; ++i)
            if (val[i] > c) { c = val[i]; k = i; }
        SWP(n_lo - 1, k);
    }
#undef SWP
    return (float)((double)fa(val[n_lo - 1], val[n_lo]) / 2.0);
}

// segment [s, s + m) of heap node h at depth `depth` (n_lo = m / 2)
__device__ __forceinline__ void ann_segment(int h, int n, int depth, int& s, int& m) {
    const int path = h + 1;
    s = 0;
    m = n;
    for (int bl = depth - 1; bl >= 0; --bl) {
        const int half = m >> 1;
        if ((path >> bl) & 1) { s += half; m -= half; }
        else m = half;
    }
}

// split node h (spread already reduced to cdim): quickselect, cut value, cell
// bounds on cdim (root rect narrowed by ancestors cutting the same dimension)
__device__ void finish_node(const Tree& t, int h, int depth, int s, int m, int cdim) {
    const int n_lo = m / 2;
    const float cvv = median_split_v(t.pidx + s, t.val + s, m, n_lo);
    float lov = t.bnd[cdim], hiv = t.bnd[t.dd + cdim];
    int a = 0;
    const int path = h + 1;
    for (int bl = depth - 1; bl >= 0; --bl) {
        const int right = (path >> bl) & 1;
        if (t.cd[a] == cdim) {
            if (right) lov = t.cv[a];
            else hiv = t.cv[a];
        }
        a = 2 * a + 1 + right;
    }
    t.cd[h] = cdim;
    t.cv[h] = cvv;
    t.lo[h] = lov;
    t.hi[h] = hiv;
}

__device__ __forceinline__ float wave_fmin(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_fmax(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

__device__ void build_par(const Tree& t) {
    const int n = t.n, dd = t.dd;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    int* pidx = t.pidx;
    for (int i = tid; i < n; i += blockDim.x) pidx[i] = i;
    __syncthreads();
    int depth = 0;
    for (int sz = n; sz >= 2; sz -= sz >> 1, ++depth) {  // sz: the level's largest segment
        const int first = (1 << depth) - 1, count = 1 << depth;
        if (sz >= kWaveSeg) {  // one wave per node
            for (int node = wave; node < count; node += nw) {
                const int h = first + node;
                int s, m;
                ann_segment(h, n, depth, s, m);
                if (m < 2) continue;
                const int* seg = pidx + s;
                int cdim = 0;
                float max_spr = 0.0f;
                for (int d = 0; d < dd; ++d) {
                    float mn = __builtin_nanf(""), mx = __builtin_nanf("");
                    for (int i = lane; i < m; i += 64) {
                        const float c = t.pts[(int64_t)seg[i] * dd + d];
                        mn = fminf(mn, c);
                        mx = fmaxf(mx, c);
                    }
                    mn = wave_fmin(mn);
                    mx = wave_fmax(mx);
                    const float c0 = t.pts[(int64_t)seg[0] * dd + d];
                    if (c0 != c0) mn = mx = c0;  // a NaN first value never moves
                    const float spr = fs(mx, mn);
                    if (spr > max_spr) { max_spr = spr; cdim = d; }
                    if (h == 0 && lane == 0) {  // annEnclRect
                        t.bnd[d] = mn;
                        t.bnd[dd + d] = mx;
                    }
                }
                for (int i = lane; i < m; i += 64) t.val[s + i] = t.pts[(int64_t)seg[i] * dd + cdim];
                __threadfence_block();  // the staged values (and bnd) before lane 0 reads them
                if (lane == 0) finish_node(t, h, depth, s, m, cdim);
            }
        } else {  // one lane per node, the reference's loops
            for (int node = tid; node < count; node += blockDim.x) {
                const int h = first + node;
                int s, m;
                ann_segment(h, n, depth, s, m);
                if (m < 2) continue;
                const int* seg = pidx + s;
                int cdim = 0;
                float max_spr = 0.0f;
                for (int d = 0; d < dd; ++d) {
                    float mn = t.pts[(int64_t)seg[0] * dd + d], mx = mn;
                    for (int i = 1; i < m; ++i) {
                        const float c = t.pts[(int64_t)seg[i] * dd + d];
                        if (c < mn) mn = c;
                        else if (c > mx) mx = c;
                    }
                    const float spr = fs(mx, mn);
                    if (spr > max_spr) { max_spr = spr; cdim = d; }
                    if (h == 0) {
                        t.bnd[d] = mn;
                        t.bnd[dd + d] = mx;
                    }
                }
                for (int i = 0; i < m; ++i) t.val[s + i] = t.pts[(int64_t)seg[i] * dd + cdim];
                finish_node(t, h, depth, s, m, cdim);
            }
        }
        __syncthreads();
    }
    if (n == 1 && tid < dd) {  // annEnclRect of a single point (no split node)
        t.bnd[tid] = t.pts[tid];
        t.bnd[dd + tid] = t.pts[tid];
    }
}

__global__ __launch_bounds__(kBuildThreads) void build_kernel(Tree t) { build_par(t); }

// one tree per workgroup: the KNNFit candidate trees of several frames
__global__ __launch_bounds__(kBuildThreads) void build_many_kernel(const Tree* __restrict__ trees) {
    build_par(trees[blockIdx.x]);
}

struct MinK {
    float* key;
    int* info;
    int k, n;
    __device__ float max_key() const { return n == k ? key[k - 1] : FLT_MAX; }
    __device__ void insert(float kv, int inf) {
        int i;
        for (i = n; i > 0; --i) {
            if (key[i - 1] > kv) { key[i] = key[i - 1]; info[i] = info[i - 1]; }
            else break;
        }
        key[i] = kv;
        info[i] = inf;
        if (n < k) ++n;
    }
};

__device__ float box_dist(const float* q, const float* lo, const float* hi, int dd) {
    float dist = 0.0f;
    for (int d = 0; d < dd; ++d) {
        if (q[d] < lo[d]) { const float t = fs(lo[d], q[d]); dist = fa(dist, fm(t, t)); }
        else if (q[d] > hi[d]) { const float t = fs(q[d], hi[d]); dist = fa(dist, fm(t, t)); }
    }
    return dist;
}

// ANNkd_leaf::ann_search: dist = dist + (q[d] - p[d])^2 with the early exit
// "some partial sum > min_dist" => not inserted.  The partial sums of
// non-negative terms only grow, so on the precomputed full distance that test
// is "dist > min_dist" -- except when the sum turns NaN, where the partial
// sums are replayed.
__device__ void leaf_visit(const Tree& t, const float* q, const float* __restrict__ dist, int p, MinK& mk) {
    const float min_dist = mk.max_key();
    const int pi = t.pidx[p];
    const float dd = dist[pi];
    bool exits;
    if (dd == dd) {
        exits = dd > min_dist;
    } else {
        const float* pp = t.pts + (int64_t)pi * t.dd;
        float s = 0.0f;
        exits = false;
        for (int d = 0; d < t.dd && !exits; ++d) {
            const float tt = fs(q[d], pp[d]);
            s = fa(s, fm(tt, tt));
            exits = s > min_dist;
        }
    }
    if (!exits) mk.insert(dd, pi);
}

// mode 0: annkSearch (DFS); mode 1: annkPriSearch (best-bin-first)
// All lanes compute the live distance of every point (sequential f32 over
// d = 0..dd-1, the leaf's own order); lane 0 then walks ANN's search over the
// stale tree with those distances.
__global__ void query_kernel(Tree t, const float* __restrict__ q, int k, int mode, float eps, int* idxs, float* errs,
                             float* dist, float* mk_key, int* mk_info, float* pq_key, int* pq_h, int* pq_s, int* pq_n) {
    for (int i = threadIdx.x; i < t.n; i += blockDim.x) {
        const float* pp = t.pts + (int64_t)i * t.dd;
        float s = 0.0f;
        for (int d = 0; d < t.dd; ++d) {
            const float tt = fs(q[d], pp[d]);
            s = fa(s, fm(tt, tt));
        }
        dist[i] = s;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    MinK mk{mk_key, mk_info, k, 0};
    const double max_err = (1.0 + (double)eps) * (1.0 + (double)eps);
    if (t.n > 0) {
        const float root_box = box_dist(q, t.bnd, t.bnd + t.dd, t.dd);
        if (mode == 0) {
            int st_h[64], st_s[64], st_n[64];
            float st_b[64];
            int sp = 0, h = 0, s = 0, n = t.n;
            float cur = root_box;
            for (;;) {
                if (n == 1) {
                    leaf_visit(t, q, dist, s, mk);
                    bool found = false;
                    while (sp > 0) {
                        --sp;
                        if ((double)st_b[sp] * max_err < (double)mk.max_key()) {
                            h = st_h[sp]; s = st_s[sp]; n = st_n[sp]; cur = st_b[sp];
                            found = true;
                            break;
                        }
                    }
                    if (!found) break;
                    continue;
                }
                const int half = n >> 1, cdim = t.cd[h];
                const float cut = fs(q[cdim], t.cv[h]);
                float bd;
                if (cut < 0.0f) {
                    bd = fs(t.lo[h], q[cdim]);
                    st_h[sp] = 2 * h + 2; st_s[sp] = s + half; st_n[sp] = n - half;
                    h = 2 * h + 1; n = half;
                } else {
                    bd = fs(q[cdim], t.hi[h]);
                    st_h[sp] = 2 * h + 1; st_s[sp] = s; st_n[sp] = half;
                    h = 2 * h + 2; s = s + half; n = n - half;
                }
                if (bd < 0.0f) bd = 0.0f;
                st_b[sp] = fa(cur, fs(fm(cut, cut), fm(bd, bd)));
                ++sp;
            }
        } else {
            int pn = 0;
            auto pq_insert = [&](float kv, int h, int s, int n) {
                int r = ++pn;
                while (r > 1) {
                    const int p = r / 2;
                    if (pq_key[p] <= kv) break;
                    pq_key[r] = pq_key[p]; pq_h[r] = pq_h[p]; pq_s[r] = pq_s[p]; pq_n[r] = pq_n[p];
                    r = p;
                }
                pq_key[r] = kv; pq_h[r] = h; pq_s[r] = s; pq_n[r] = n;
            };
            pq_insert(root_box, 0, 0, t.n);
            while (pn > 0) {
                const float box = pq_key[1];
                int h = pq_h[1], s = pq_s[1], n = pq_n[1];
                {
                    const float kn = pq_key[pn];
                    const int lh = pq_h[pn], ls = pq_s[pn], ln = pq_n[pn];
                    --pn;
                    int p = 1, r = 2;
                    while (r <= pn) {
                        if (r < pn && pq_key[r] > pq_key[r + 1]) ++r;
                        if (kn <= pq_key[r]) break;
                        pq_key[p] = pq_key[r]; pq_h[p] = pq_h[r]; pq_s[p] = pq_s[r]; pq_n[p] = pq_n[r];
                        p = r;
                        r = p << 1;
                    }
                    pq_key[p] = kn; pq_h[p] = lh; pq_s[p] = ls; pq_n[p] = ln;
                }
                if ((double)box * max_err >= (double)mk.max_key()) break;
                for (;;) {
                    if (n == 1) {
                        leaf_visit(t, q, dist, s, mk);
                        break;
                    }
                    const int half = n >> 1, cdim = t.cd[h];
                    const float cut = fs(q[cdim], t.cv[h]);
                    float bd;
                    int nh, ns, nn, fh, fs_, fn;
                    if (cut < 0.0f) {
                        bd = fs(t.lo[h], q[cdim]);
                        nh = 2 * h + 1; ns = s; nn = half;
                        fh = 2 * h + 2; fs_ = s + half; fn = n - half;
                    } else {
                        bd = fs(q[cdim], t.hi[h]);
                        nh = 2 * h + 2; ns = s + half; nn = n - half;
                        fh = 2 * h + 1; fs_ = s; fn = half;
                    }
                    if (bd < 0.0f) bd = 0.0f;
                    pq_insert(fa(box, fs(fm(cut, cut), fm(bd, bd))), fh, fs_, fn);
                    h = nh; s = ns; n = nn;
                }
            }
        }
    }
    for (int i = 0; i < k; ++i) {
        errs[i] = i < mk.n ? mk.key[i] : FLT_MAX;
        idxs[i] = i < mk.n ? mk.info[i] : -1;
    }
}


// ---------------------------------------------------------------------------
// TFrame.KNNFit for the queries whose tie set exceeds the 64-NN bucket
// (encoder.lpr:945-958): ANN's priority search (annkPriSearch @0x180011da0,
// k = 64, eps = 0) over the frame's kd-tree of the 4R candidates, exactly as
// the DLL runs it -- best-bin-first order, the stable ANNmin_k insert -- so
// which of the equal-distance candidates fill the bucket, and then the
// smallest index among the bucket's near-ties, follow the reference.  One
// thread per query; the bucket lives in LDS, the box queue in HBM.
// ---------------------------------------------------------------------------
using OvJob = gsc::KnnOvJob;

constexpr int kOvBlock = 64;
constexpr int kBucket = 64;  // CBucketSize (encoder.lpr:917)

__global__ __launch_bounds__(kOvBlock) void knnfit_ann_kernel(const Tree* __restrict__ trees,
                                                               const OvJob* __restrict__ jobs, int njobs,
                                                               const float* __restrict__ qall, int* __restrict__ out,
                                                               float* __restrict__ pq_key, int4* __restrict__ pq_node,
                                                               int pq_cap) {
    __shared__ float s_key[kOvBlock][kBucket + 1];
    __shared__ int s_info[kOvBlock][kBucket + 1];
    const int j = blockIdx.x * kOvBlock + threadIdx.x;
    if (j >= njobs) return;
    const OvJob job = jobs[j];
    const Tree t = trees[job.tree];
    const float* q = qall + job.q_off;
    MinK mk{s_key[threadIdx.x], s_info[threadIdx.x], kBucket, 0};
    float* pk = pq_key + (int64_t)j * pq_cap;
    int4* pn_ = pq_node + (int64_t)j * pq_cap;
    int pn = 0;
    auto pq_insert = [&](float kv, int h, int s, int n) {  // ANNpr_queue::insert (sift up, stop at <=)
        int r = ++pn;
        while (r > 1) {
            const int p = r / 2;
            if (pk[p] <= kv) break;
            pk[r] = pk[p];
            pn_[r] = pn_[p];
            r = p;
        }
        pk[r] = kv;
        pn_[r] = make_int4(h, s, n, 0);
    };
    if (t.n > 0) {
        pq_insert(box_dist(q, t.bnd, t.bnd + t.dd, t.dd), 0, 0, t.n);
        while (pn > 0) {
            const float box = pk[1];
            const int4 nd = pn_[1];
            {  // extract_min: last element sifted down (child r+1 iff key[r] > key[r+1]; stop at kn <= key[r])
                const float kn = pk[pn];
                const int4 ln = pn_[pn];
                --pn;
                int p = 1, r = 2;
                while (r <= pn) {
                    if (r < pn && pk[r] > pk[r + 1]) ++r;
                    if (kn <= pk[r]) break;
                    pk[p] = pk[r];
                    pn_[p] = pn_[r];
                    p = r;
                    r = p << 1;
                }
                pk[p] = kn;
                pn_[p] = ln;
            }
            if ((double)box >= (double)mk.max_key()) break;  // box * (1 + eps)^2, eps = 0
            int h = nd.x, s = nd.y, n = nd.z;
            for (;;) {  // ANNkd_split::ann_pri_search: push the far child, descend the near one
                // bounds check (the replay's arrays are poison-filled, gsc_runtime.cpp
                // DevArena): a node, segment or point index outside its tree's
                // arrays reports -4 instead of reading another frame's memory
                if (s < 0 || n < 1 || s + n > t.n || (t.ncap > 0 && (h < 0 || h >= t.ncap))) {
                    out[job.out] = -4;
                    return;
                }
                if (n == 1) {
                    const float min_dist = mk.max_key();
                    const int pi = t.pidx[s];
                    if (pi < 0 || pi >= t.n) {
                        out[job.out] = -4;
                        return;
                    }
                    const float* pp = t.pts + (int64_t)pi * t.dd;
                    float dist = 0.0f;
                    int d;
                    for (d = 0; d < t.dd; ++d) {
                        const float tt = fs(q[d], pp[d]);
                        if ((dist = fa(dist, fm(tt, tt))) > min_dist) break;
                    }
                    if (d >= t.dd) mk.insert(dist, pi);
                    break;
                }
                const int half = n >> 1, cdim = t.cd[h];
                if (cdim < 0 || cdim >= t.dd) {  // an unbuilt node (poison -1)
                    out[job.out] = -4;
                    return;
                }
                const float cut = fs(q[cdim], t.cv[h]);
                float bd;
                int nh, ns, nn, fh, fs_, fn;
                if (cut < 0.0f) {
                    bd = fs(t.lo[h], q[cdim]);
                    nh = 2 * h + 1; ns = s; nn = half;
                    fh = 2 * h + 2; fs_ = s + half; fn = n - half;
                } else {
                    bd = fs(q[cdim], t.hi[h]);
                    nh = 2 * h + 2; ns = s + half; nn = n - half;
                    fh = 2 * h + 1; fs_ = s; fn = half;
                }
                if (bd < 0.0f) bd = 0.0f;
                if (pn + 1 >= pq_cap) {  // cannot happen: at most one push per split node
                    out[job.out] = -3;
                    return;
                }
                pq_insert(fa(box, fs(fm(cut, cut), fm(bd, bd))), fh, fs_, fn);
                h = nh; s = ns; n = nn;
            }
        }
    }
    // tie rule (encoder.lpr:954-958): the smallest index among the bucket's
    // entries whose sqrt(err / CS) is SameValue with the first one's
    const float csf = (float)t.dd;
    int b = mk.n > 0 ? mk.info[0] : -1;
    const float s0 = mk.n > 0 ? sqrt_rn(mk.key[0] / csf) : 0.0f;
    for (int i = 0; i < mk.n; ++i) {
        const int id = mk.info[i];
        if (id >= 0 && id <= b - 1) {
            const float sj = sqrt_rn(mk.key[i] / csf);
            const float dl = s0 > sj ? fs(s0, sj) : fs(sj, s0);
            if (dl <= job.eps) b = id;
        }
    }
    out[job.out] = b;
}
}  // namespace ann
}  // namespace gsc

// val: n floats of scratch
extern "C" hipError_t gsc_launch_ann_build(const float* pts, int n, int dd, int* pidx, int* cd, float* cv, float* lo,
                                           float* hi, float* bnd, float* val, hipStream_t st) {
    gsc::ann::Tree t{pts, n, dd, pidx, cd, cv, lo, hi, bnd, val};
    hipLaunchKernelGGL(gsc::ann::build_kernel, dim3(1), dim3(gsc::ann::kBuildThreads), 0, st, t);
    return hipGetLastError();
}

extern "C" hipError_t gsc_launch_ann_query(const float* pts, int n, int dd, int* pidx, int* cd, float* cv, float* lo,
                                           float* hi, float* bnd, const float* q, int k, int mode, float eps, int* idxs,
                                           float* errs, float* dist, float* mk_key, int* mk_info, float* pq_key,
                                           int* pq_h, int* pq_s, int* pq_n, hipStream_t st) {
    gsc::ann::Tree t{pts, n, dd, pidx, cd, cv, lo, hi, bnd, nullptr};
    hipLaunchKernelGGL(gsc::ann::query_kernel, dim3(1), dim3(1024), 0, st, t, q, k, mode, eps, idxs, errs, dist, mk_key,
                       mk_info, pq_key, pq_h, pq_s, pq_n);
    return hipGetLastError();
}

// trees: device array of ntrees descriptors (their arrays already allocated)
extern "C" hipError_t gsc_launch_ann_build_many(const void* trees, int ntrees, hipStream_t st) {
    hipLaunchKernelGGL(gsc::ann::build_many_kernel, dim3(ntrees), dim3(gsc::ann::kBuildThreads), 0, st,
                       static_cast<const gsc::ann::Tree*>(trees));
    return hipGetLastError();
}


extern "C" hipError_t gsc_launch_knnfit_ann(const void* trees, const void* jobs, int njobs, const float* q, int* out,
                                            float* pq_key, void* pq_node, int pq_cap, hipStream_t st) {
    const int blocks = (njobs + gsc::ann::kOvBlock - 1) / gsc::ann::kOvBlock;
    hipLaunchKernelGGL(gsc::ann::knnfit_ann_kernel, dim3(blocks), dim3(gsc::ann::kOvBlock), 0, st,
                       static_cast<const gsc::ann::Tree*>(trees), static_cast<const gsc::ann::OvJob*>(jobs), njobs, q,
                       out, pq_key, static_cast<int4*>(pq_node), pq_cap);
    return hipGetLastError();
}
