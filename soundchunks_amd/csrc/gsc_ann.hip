// GPU implementation of the ANN.dll surface bound by extern.pas:118-123
// (ann_kdtree_create / _search / _pri_search / _search_multi /
// _pri_search_multi).  The encoder itself uses the batched kernels in
// gsc_kernels.hip; this file serves the per-query drop-in ABI, so it favours
// exactness over speed: one lane runs ANN 1.1's sequential build and search
// code (ANN.dll @0x180014620 ctor, @0x1800124b0 annkSearch,
// @0x180011da0 annkPriSearch) on device memory.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

namespace gsc {
namespace ann {

struct Tree {
    const float* pts;  // n * dd, row major (the live point values)
    int n, dd;
    int* pidx;         // n
    int* cd;           // heap-indexed split data, 2 * pow2ceil(n) entries
    float* cv;
    float* lo;
    float* hi;
    float* bnd;        // 2 * dd: bounding rect lo | hi
};

__device__ __forceinline__ float fa(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fs(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ float fm(float a, float b) { return __fmul_rn(a, b); }

#define PA(i, d) (t.pts[(int64_t)pidx[(i)] * t.dd + (d)])

__device__ void median_split(const Tree& t, int* pidx, int n, int d, float* cv, int n_lo) {
    int l = 0, r = n - 1;
#define SWP(a, b) { const int x_ = pidx[a]; pidx[a] = pidx[b]; pidx[b] = x_; }
    while (l < r) {
        int i = (r + l) / 2, k;
        if (PA(i, d) > PA(r, d)) SWP(i, r)
        SWP(l, i);
        const float c = PA(l, d);
        i = l;
        k = r;
        for (;;) {
            while (PA(++i, d) < c) {}
            while (PA(--k, d) > c) {}
            if (i < k) SWP(i, k) else break;
        }
        SWP(l, k);
        if (k > n_lo) r = k - 1;
        else if (k < n_lo) l = k + 1;
        else break;
    }
    if (n_lo > 0) {
        float c = PA(0, d);
        int k = 0;
        for (int i = 1; i < n_lo; ++i)
            if (PA(i, d) > c) { c = PA(i, d); k = i; }
        SWP(n_lo - 1, k);
    }
#undef SWP
    *cv = (float)((double)fa(PA(n_lo - 1, d), PA(n_lo, d)) / 2.0);
}

// ANNkd_tree ctor with ANN_KD_STD, bs = 1: annEnclRect, then rkd_tree with
// kd_split (annMaxSpread + annMedianSplit) -- iterative pre-order
__global__ void build_kernel(Tree t) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int n = t.n, dd = t.dd;
    for (int i = 0; i < n; ++i) t.pidx[i] = i;
    int* pidx = t.pidx;
    for (int d = 0; d < dd; ++d) {
        float lo = PA(0, d), hi = PA(0, d);
        for (int i = 0; i < n; ++i) {
            const float v = PA(i, d);
            if (v < lo) lo = v;
            else if (v > hi) hi = v;
        }
        t.bnd[d] = lo;
        t.bnd[dd + d] = hi;
    }
    // explicit stack of (heap index, segment start, size); bounds per node are
    // the root rect narrowed by ancestors cutting the same dimension
    int st_h[64], st_s[64], st_n[64];
    int sp = 0;
    st_h[0] = 0; st_s[0] = 0; st_n[0] = n; sp = 1;
    while (sp > 0) {
        --sp;
        const int h = st_h[sp], s = st_s[sp], m = st_n[sp];
        if (m < 2) continue;
        int* seg = t.pidx + s;
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
        }
        const int n_lo = m / 2;
        float cvv;
        median_split(t, seg, m, cdim, &cvv, n_lo);
        float lov = t.bnd[cdim], hiv = t.bnd[dd + cdim];
        {
            int a = 0;
            const int path = h + 1;
            const int depth = 31 - __clz(path);
            for (int bl = depth - 1; bl >= 0; --bl) {
                const int right = (path >> bl) & 1;
                if (t.cd[a] == cdim) {
                    if (right) lov = t.cv[a];
                    else hiv = t.cv[a];
                }
                a = 2 * a + 1 + right;
            }
        }
        t.cd[h] = cdim;
        t.cv[h] = cvv;
        t.lo[h] = lov;
        t.hi[h] = hiv;
        // pre-order: push hi first so lo is processed first
        st_h[sp] = 2 * h + 2; st_s[sp] = s + n_lo; st_n[sp] = m - n_lo; ++sp;
        st_h[sp] = 2 * h + 1; st_s[sp] = s; st_n[sp] = n_lo; ++sp;
    }
}
#undef PA

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

__device__ void leaf_visit(const Tree& t, const float* q, int p, MinK& mk) {
    const float min_dist = mk.max_key();
    const float* pp = t.pts + (int64_t)t.pidx[p] * t.dd;
    float dist = 0.0f;
    int d;
    for (d = 0; d < t.dd; ++d) {
        const float tt = fs(q[d], pp[d]);
        if ((dist = fa(dist, fm(tt, tt))) > min_dist) break;
    }
    if (d >= t.dd) mk.insert(dist, t.pidx[p]);
}

// mode 0: annkSearch (DFS); mode 1: annkPriSearch (best-bin-first)
__global__ void query_kernel(Tree t, const float* __restrict__ q, int k, int mode, float eps, int* idxs, float* errs,
                             float* mk_key, int* mk_info, float* pq_key, int* pq_h, int* pq_s, int* pq_n) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
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
                    leaf_visit(t, q, s, mk);
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
                        leaf_visit(t, q, s, mk);
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

}  // namespace ann
}  // namespace gsc

extern "C" hipError_t gsc_launch_ann_build(const float* pts, int n, int dd, int* pidx, int* cd, float* cv, float* lo,
                                           float* hi, float* bnd, hipStream_t st) {
    gsc::ann::Tree t{pts, n, dd, pidx, cd, cv, lo, hi, bnd};
    hipLaunchKernelGGL(gsc::ann::build_kernel, dim3(1), dim3(64), 0, st, t);
    return hipGetLastError();
}

extern "C" hipError_t gsc_launch_ann_query(const float* pts, int n, int dd, int* pidx, int* cd, float* cv, float* lo,
                                           float* hi, float* bnd, const float* q, int k, int mode, float eps, int* idxs,
                                           float* errs, float* mk_key, int* mk_info, float* pq_key, int* pq_h,
                                           int* pq_s, int* pq_n, hipStream_t st) {
    gsc::ann::Tree t{pts, n, dd, pidx, cd, cv, lo, hi, bnd};
    hipLaunchKernelGGL(gsc::ann::query_kernel, dim3(1), dim3(64), 0, st, t, q, k, mode, eps, idxs, errs, mk_key,
                       mk_info, pq_key, pq_h, pq_s, pq_n);
    return hipGetLastError();
}
