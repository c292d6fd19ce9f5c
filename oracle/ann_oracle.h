/*
 * ORACLE (test infrastructure only) -- CPU restatement of the ANN 1.1.x
 * kd-tree that reference encoder/ANN.dll exports:
 *   ann_kdtree_create  @0x180003c50 -> ANNkd_tree ctor @0x180014620
 *     (annEnclRect @0x180014980, kd_split = annMaxSpread @0x180015260 +
 *      annMedianSplit @0x180015680, rkd_tree @0x180014420)
 *   ann_kdtree_search  @0x180003cd0 -> annkSearch @0x1800124b0
 *   ann_kdtree_pri_search_multi @0x180003db0 -> annkPriSearch @0x180011da0
 * Third-party dependency: ANN 1.1.x (Mount & Arya), float coordinates,
 * re-entrant fork; un-vendored, no source under /root/reference.
 * The tree keeps the caller's row pointers (no copy): searches read the
 * *current* point values, exactly like the DLL (encoder.lpr:729-745 relies
 * on it).  Parity against the real DLL is unpinned (the DLL cannot run here).
 */
#ifndef GSC_ORACLE_ANN_H
#define GSC_ORACLE_ANN_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ora_kdtree ora_kdtree;

ora_kdtree *ora_kdtree_create(float **pa, int n, int dd, int bs);
void ora_kdtree_destroy(ora_kdtree *t);
/* exact (eps = 0) standard k = 1 search; returns index, *err = squared dist */
int ora_kdtree_search(ora_kdtree *t, const float *q, float eps, float *err);
/* priority search, k = cnt */
void ora_kdtree_pri_search_multi(ora_kdtree *t, int *idxs, float *errs, int cnt, const float *q,
                                 float eps);
void ora_kdtree_search_multi(ora_kdtree *t, int *idxs, float *errs, int cnt, const float *q,
                             float eps);

/* introspection for tests / GPU parity: node arrays in pre-order.
 * For node i: leaf_pt[i] >= 0 => leaf holding that point (bs = 1),
 * else split with cut_dim/cut_val/lo/hi and children lo_child/hi_child. */
int ora_kdtree_node_count(const ora_kdtree *t);
void ora_kdtree_export(const ora_kdtree *t, int *cut_dim, float *cut_val, float *lo_bnd,
                       float *hi_bnd, int *lo_child, int *hi_child, int *leaf_pt);
/* statistics of the last search (leaves visited, split nodes visited) */
void ora_kdtree_last_stats(const ora_kdtree *t, long *leaves, long *splits);

#ifdef __cplusplus
}
#endif
#endif
