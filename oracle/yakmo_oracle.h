/*
 * ORACLE (test infrastructure only) -- CPU restatement of the part of
 * reference encoder/yakmo_single.dll (yakmo k-means, Naoki Yoshinaga, VS2017
 * build, C-API fork; no source in /root/reference) that reaches the .gsc.
 *
 * encoder.lpr:824-828 calls yakmo_create(K,1,0,1,0,0,v): k-means++ seeding
 * with the fixed xorshift128 seeds, then one Lloyd pass (maxIter = 0).
 * Only the returned centroids survive (KNNScanReduce overwrites the labels,
 * encoder.lpr:742), and those are the means of the *seeding* assignment
 * (SURVEY.md 8a row a2, App. C.1).  Restated from the disassembly:
 *   seeding          yakmo_single.dll @0x1800016f0..0x180001f7e
 *     RNG            @0x1800018c4 (x<<11, w>>19, t>>8), draw = f32(f64(w)*2^-64)
 *     first pick     @0x18000193a floorf(r*f32(N))
 *     lower_bound    @0x1800019d0 (count halving, r*total > cum[mid] moves right)
 *     collision      @0x180001b20 (idx+1 wrap to 0), clamp @0x180001c50
 *     distance       @0x180001dc0 d = ((c.norm + x.norm) + 0) then d -= (x+x)*c
 *     d0/d1/id       @0x180001e1d, cum prefix @0x180001e74
 *   centroid update  @0x180002290 c = sum / f32(count)
 *   point norm       @0x1800015cb norm += v*v (f32, in order)
 * Labels returned by ora_yakmo_train are the seeding assignment (the dead
 * Lloyd reassignment is not restated; documented in DESIGN.md).
 * Parity against the real DLL is unpinned (it cannot run here).
 */
#ifndef GSC_ORACLE_YAKMO_H
#define GSC_ORACLE_YAKMO_H

#ifdef __cplusplus
extern "C" {
#endif

/* X: N rows of D floats (row-major).  Writes K*D centroids and N labels.
 * Returns 0 on success, -1 if K >= N (the DLL would spin forever). */
int ora_yakmo_seed_means(int N, int D, const float *X, int K, float *centroids, int *labels);

#ifdef __cplusplus
}
#endif
#endif
