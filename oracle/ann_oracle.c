/*
 * ORACLE (test infrastructure only) -- ANN 1.1.x kd-tree restatement.
 * See ann_oracle.h.  float coordinates and float distances throughout
 * (TANNFloat = Single, extern.pas:68), maxErr = (1 + eps)^2 in double.
 */
#include "ann_oracle.h"

#include <float.h>
#include <stdlib.h>
#include <string.h>

#define ANN_DIST_INF FLT_MAX /* ANN.dll VA 0x1800b88cc */

typedef struct {
    int cut_dim;
    float cut_val, lo, hi;
    int child[2]; /* node indices; -1 = KD_TRIVIAL */
    int n_pts;    /* > 0 => leaf */
    int bkt;      /* offset into the tree's pidx for leaves */
} node_t;

struct ora_kdtree {
    float **pts;
    int n, dim, bs;
    int *pidx;
    float *bnd_lo, *bnd_hi;
    node_t *nodes;
    int n_nodes, cap_nodes;
    int root; /* -1 => KD_TRIVIAL */
    long st_leaves, st_splits;
};

#define PA(i, d) (pa[pidx[(i)]][(d)])
#define PASWAP(a, b) { int tmp_ = pidx[a]; pidx[a] = pidx[b]; pidx[b] = tmp_; }

static void encl_rect(float **pa, const int *pidx, int n, int dim, float *lo, float *hi) {
    for (int d = 0; d < dim; d++) {
        float lo_bnd = PA(0, d), hi_bnd = PA(0, d);
        for (int i = 0; i < n; i++) {
            if (PA(i, d) < lo_bnd) lo_bnd = PA(i, d);
            else if (PA(i, d) > hi_bnd) hi_bnd = PA(i, d);
        }
        lo[d] = lo_bnd;
        hi[d] = hi_bnd;
    }
}

static float spread(float **pa, const int *pidx, int n, int d) {
    float mn = PA(0, d), mx = PA(0, d);
    for (int i = 1; i < n; i++) {
        float c = PA(i, d);
        if (c < mn) mn = c;
        else if (c > mx) mx = c;
    }
    return mx - mn;
}

static int max_spread(float **pa, const int *pidx, int n, int dim) {
    int max_dim = 0;
    float max_spr = 0;
    if (n == 0) return max_dim;
    for (int d = 0; d < dim; d++) {
        float spr = spread(pa, pidx, n, d);
        if (spr > max_spr) { max_spr = spr; max_dim = d; }
    }
    return max_dim;
}

static void median_split(float **pa, int *pidx, int n, int d, float *cv, int n_lo) {
    int l = 0, r = n - 1;
    while (l < r) {
        int i = (r + l) / 2;
        int k;
        if (PA(i, d) > PA(r, d)) PASWAP(i, r)
        PASWAP(l, i);
        float c = PA(l, d);
        i = l;
        k = r;
        for (;;) {
            while (PA(++i, d) < c) {}
            while (PA(--k, d) > c) {}
            if (i < k) PASWAP(i, k) else break;
        }
        PASWAP(l, k);
        if (k > n_lo) r = k - 1;
        else if (k < n_lo) l = k + 1;
        else break;
    }
    if (n_lo > 0) {
        float c = PA(0, d);
        int k = 0;
        for (int i = 1; i < n_lo; i++) {
            if (PA(i, d) > c) { c = PA(i, d); k = i; }
        }
        PASWAP(n_lo - 1, k);
    }
    *cv = (float)((double)(PA(n_lo - 1, d) + PA(n_lo, d)) / 2.0);
}

static int new_node(ora_kdtree *t) {
    if (t->n_nodes == t->cap_nodes) {
        t->cap_nodes = t->cap_nodes ? t->cap_nodes * 2 : 64;
        t->nodes = (node_t *)realloc(t->nodes, sizeof(node_t) * (size_t)t->cap_nodes);
    }
    memset(&t->nodes[t->n_nodes], 0, sizeof(node_t));
    return t->n_nodes++;
}

/* rkd_tree: pre-order node allocation (split node allocated before children,
 * which is how GPU code lays the tree out; ANN allocates it after, which does
 * not change semantics). */
static int rkd(ora_kdtree *t, int *pidx, int n, float *blo, float *bhi) {
    if (n <= t->bs) {
        if (n == 0) return -1;
        int id = new_node(t);
        t->nodes[id].n_pts = n;
        t->nodes[id].bkt = (int)(pidx - t->pidx);
        return id;
    }
    int cd, n_lo;
    float cv;
    cd = max_spread(t->pts, pidx, n, t->dim);
    n_lo = n / 2;
    median_split(t->pts, pidx, n, cd, &cv, n_lo);
    int id = new_node(t);
    float lv = blo[cd], hv = bhi[cd];
    bhi[cd] = cv;
    int lo = rkd(t, pidx, n_lo, blo, bhi);
    bhi[cd] = hv;
    blo[cd] = cv;
    int hi = rkd(t, pidx + n_lo, n - n_lo, blo, bhi);
    blo[cd] = lv;
    node_t *nd = &t->nodes[id];
    nd->cut_dim = cd;
    nd->cut_val = cv;
    nd->lo = lv;
    nd->hi = hv;
    nd->child[0] = lo;
    nd->child[1] = hi;
    nd->n_pts = 0;
    return id;
}

ora_kdtree *ora_kdtree_create(float **pa, int n, int dd, int bs) {
    ora_kdtree *t = (ora_kdtree *)calloc(1, sizeof(ora_kdtree));
    t->pts = pa;
    t->n = n;
    t->dim = dd;
    t->bs = bs;
    t->pidx = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) t->pidx[i] = i;
    t->bnd_lo = (float *)calloc((size_t)dd, sizeof(float));
    t->bnd_hi = (float *)calloc((size_t)dd, sizeof(float));
    t->root = -1;
    if (n == 0) return t;
    encl_rect(pa, t->pidx, n, dd, t->bnd_lo, t->bnd_hi);
    float *blo = (float *)malloc(sizeof(float) * (size_t)dd);
    float *bhi = (float *)malloc(sizeof(float) * (size_t)dd);
    memcpy(blo, t->bnd_lo, sizeof(float) * (size_t)dd);
    memcpy(bhi, t->bnd_hi, sizeof(float) * (size_t)dd);
    t->root = rkd(t, t->pidx, n, blo, bhi);
    free(blo);
    free(bhi);
    return t;
}

void ora_kdtree_destroy(ora_kdtree *t) {
    if (!t) return;
    free(t->pidx);
    free(t->bnd_lo);
    free(t->bnd_hi);
    free(t->nodes);
    free(t);
}

/* ---- ANNmin_k ----------------------------------------------------------- */
typedef struct {
    float key;
    int info;
} mk_node;
typedef struct {
    int k, n;
    mk_node *mk;
} min_k;

static inline float mk_max_key(const min_k *m) { return m->n == m->k ? m->mk[m->k - 1].key : ANN_DIST_INF; }
static inline void mk_insert(min_k *m, float kv, int inf) {
    int i;
    for (i = m->n; i > 0; i--) {
        if (m->mk[i - 1].key > kv) m->mk[i] = m->mk[i - 1];
        else break;
    }
    m->mk[i].key = kv;
    m->mk[i].info = inf;
    if (m->n < m->k) m->n++;
}

static float box_distance(const float *q, const float *lo, const float *hi, int dim) {
    float dist = 0.0f, t;
    for (int d = 0; d < dim; d++) {
        if (q[d] < lo[d]) { t = lo[d] - q[d]; dist = dist + t * t; }
        else if (q[d] > hi[d]) { t = q[d] - hi[d]; dist = dist + t * t; }
    }
    return dist;
}

typedef struct {
    ora_kdtree *t;
    const float *q;
    double max_err;
    min_k *mk;
} sctx;

static void leaf_search(sctx *c, const node_t *nd) {
    ora_kdtree *t = c->t;
    float min_dist = mk_max_key(c->mk);
    for (int i = 0; i < nd->n_pts; i++) {
        int pi = t->pidx[nd->bkt + i];
        const float *pp = t->pts[pi];
        float dist = 0.0f;
        int d;
        for (d = 0; d < t->dim; d++) {
            float tt = c->q[d] - pp[d];
            if ((dist = dist + tt * tt) > min_dist) break;
        }
        if (d >= t->dim) {
            mk_insert(c->mk, dist, pi);
            min_dist = mk_max_key(c->mk);
        }
    }
    t->st_leaves++;
}

static void split_search(sctx *c, int id, float box_dist) {
    if (id < 0) return; /* KD_TRIVIAL: nothing */
    const node_t *nd = &c->t->nodes[id];
    if (nd->n_pts > 0) { leaf_search(c, nd); return; }
    c->t->st_splits++;
    float cut_diff = c->q[nd->cut_dim] - nd->cut_val;
    if (cut_diff < 0) {
        split_search(c, nd->child[0], box_dist);
        float box_diff = nd->lo - c->q[nd->cut_dim];
        if (box_diff < 0) box_diff = 0;
        box_dist = box_dist + (cut_diff * cut_diff - box_diff * box_diff);
        if ((double)box_dist * c->max_err < (double)mk_max_key(c->mk)) split_search(c, nd->child[1], box_dist);
    } else {
        split_search(c, nd->child[1], box_dist);
        float box_diff = c->q[nd->cut_dim] - nd->hi;
        if (box_diff < 0) box_diff = 0;
        box_dist = box_dist + (cut_diff * cut_diff - box_diff * box_diff);
        if ((double)box_dist * c->max_err < (double)mk_max_key(c->mk)) split_search(c, nd->child[0], box_dist);
    }
}

void ora_kdtree_search_multi(ora_kdtree *t, int *idxs, float *errs, int cnt, const float *q, float eps) {
    min_k mk;
    mk.k = cnt;
    mk.n = 0;
    mk.mk = (mk_node *)malloc(sizeof(mk_node) * (size_t)(cnt + 1));
    sctx c = {t, q, (1.0 + (double)eps) * (1.0 + (double)eps), &mk};
    t->st_leaves = t->st_splits = 0;
    if (t->root >= 0) split_search(&c, t->root, box_distance(q, t->bnd_lo, t->bnd_hi, t->dim));
    for (int i = 0; i < cnt; i++) {
        errs[i] = i < mk.n ? mk.mk[i].key : ANN_DIST_INF;
        idxs[i] = i < mk.n ? mk.mk[i].info : -1;
    }
    free(mk.mk);
}

int ora_kdtree_search(ora_kdtree *t, const float *q, float eps, float *err) {
    int idx;
    float e;
    ora_kdtree_search_multi(t, &idx, &e, 1, q, eps);
    if (err) *err = e;
    return idx;
}

/* ---- ANNpr_queue (1-indexed binary heap) -------------------------------- */
typedef struct {
    float key;
    int info;
} pq_node;

void ora_kdtree_pri_search_multi(ora_kdtree *t, int *idxs, float *errs, int cnt, const float *q, float eps) {
    min_k mk;
    mk.k = cnt;
    mk.n = 0;
    mk.mk = (mk_node *)malloc(sizeof(mk_node) * (size_t)(cnt + 1));
    double max_err = (1.0 + (double)eps) * (1.0 + (double)eps);
    int max_size = t->n;
    pq_node *pq = (pq_node *)malloc(sizeof(pq_node) * (size_t)(max_size + 2));
    int pn = 0;
    t->st_leaves = t->st_splits = 0;
#define PQ_INSERT(kv_, inf_)                                 \
    do {                                                     \
        float kv = (kv_);                                    \
        int r = ++pn;                                        \
        while (r > 1) {                                      \
            int p = r / 2;                                   \
            if (pq[p].key <= kv) break;                      \
            pq[r] = pq[p];                                   \
            r = p;                                           \
        }                                                    \
        pq[r].key = kv;                                      \
        pq[r].info = (inf_);                                 \
    } while (0)
    if (t->root >= 0) {
        PQ_INSERT(box_distance(q, t->bnd_lo, t->bnd_hi, t->dim), t->root);
        while (pn > 0) {
            float box_dist = pq[1].key;
            int np = pq[1].info;
            {
                float kn = pq[pn--].key;
                int p = 1, r = 2;
                while (r <= pn) {
                    if (r < pn && pq[r].key > pq[r + 1].key) r++;
                    if (kn <= pq[r].key) break;
                    pq[p] = pq[r];
                    p = r;
                    r = p << 1;
                }
                pq[p] = pq[pn + 1];
            }
            if ((double)box_dist * max_err >= (double)mk_max_key(&mk)) break;
            /* node->ann_pri_search(box_dist): descend near children, push far */
            int id = np;
            for (;;) {
                const node_t *nd = &t->nodes[id];
                if (nd->n_pts > 0) {
                    float min_dist = mk_max_key(&mk);
                    for (int i = 0; i < nd->n_pts; i++) {
                        int pi = t->pidx[nd->bkt + i];
                        const float *pp = t->pts[pi];
                        float dist = 0.0f;
                        int d;
                        for (d = 0; d < t->dim; d++) {
                            float tt = q[d] - pp[d];
                            if ((dist = dist + tt * tt) > min_dist) break;
                        }
                        if (d >= t->dim) {
                            mk_insert(&mk, dist, pi);
                            min_dist = mk_max_key(&mk);
                        }
                    }
                    t->st_leaves++;
                    break;
                }
                t->st_splits++;
                float cut_diff = q[nd->cut_dim] - nd->cut_val;
                float box_diff, new_dist;
                int near, far;
                if (cut_diff < 0) {
                    box_diff = nd->lo - q[nd->cut_dim];
                    near = nd->child[0];
                    far = nd->child[1];
                } else {
                    box_diff = q[nd->cut_dim] - nd->hi;
                    near = nd->child[1];
                    far = nd->child[0];
                }
                if (box_diff < 0) box_diff = 0;
                new_dist = box_dist + (cut_diff * cut_diff - box_diff * box_diff);
                if (far >= 0) PQ_INSERT(new_dist, far);
                if (near < 0) break; /* KD_TRIVIAL near child: nothing to search */
                id = near;
            }
        }
    }
#undef PQ_INSERT
    for (int i = 0; i < cnt; i++) {
        errs[i] = i < mk.n ? mk.mk[i].key : ANN_DIST_INF;
        idxs[i] = i < mk.n ? mk.mk[i].info : -1;
    }
    free(pq);
    free(mk.mk);
}

int ora_kdtree_node_count(const ora_kdtree *t) { return t->n_nodes; }

void ora_kdtree_export(const ora_kdtree *t, int *cut_dim, float *cut_val, float *lo_bnd, float *hi_bnd,
                       int *lo_child, int *hi_child, int *leaf_pt) {
    for (int i = 0; i < t->n_nodes; i++) {
        const node_t *nd = &t->nodes[i];
        cut_dim[i] = nd->cut_dim;
        cut_val[i] = nd->cut_val;
        lo_bnd[i] = nd->lo;
        hi_bnd[i] = nd->hi;
        lo_child[i] = nd->child[0];
        hi_child[i] = nd->child[1];
        leaf_pt[i] = nd->n_pts > 0 ? t->pidx[nd->bkt] : -1;
    }
}

void ora_kdtree_last_stats(const ora_kdtree *t, long *leaves, long *splits) {
    if (leaves) *leaves = t->st_leaves;
    if (splits) *splits = t->st_splits;
}
