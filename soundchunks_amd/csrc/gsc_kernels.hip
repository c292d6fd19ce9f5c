// SoundChunks encode hot path on MI355X (gfx950): hand-written HIP kernels.
//
//   scan_pass_kernel    TFrame.KNNScanReduce over ANN's stale kd-tree, one
//                       search at a time (encoder.lpr:699-765; ANN.dll App.
//                       C.2), one CU / frame: the generic path for shapes and
//                       passes the batched kernel (gsc_scan.hip) does not take
//   (yakmo seeding: gsc_yakmo.hip)
//   knnfit_kernel       TFrame.KNNFit 64-NN + tie rule (encoder.lpr:915-965)
//
// Everything is bit-exact with the reference's SSE scalar arithmetic: no FMA
// (built with -ffp-contract=off), IEEE f32 division/sqrt, sequential
// reduction order wherever the reference is sequential.  No MFMA: the
// distance sums must round term by term exactly like subss/mulss/addss.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "gsc_device.h"
#include "gsc_tree.h"

namespace gsc {


// ============================================================================
// KNNScanReduce with exact emulation of ANN's stale kd-tree search.
//
// Per pass: rebuild the ANN tree (ANN_KD_STD, bs = 1) over the centroids
// exactly as annMaxSpread/annMedianSplit would, then for every point in
// order: nearest by ANN DFS over the *stale* tree with *live* centroids,
// online update of that centroid.  The 4096 centroids sit in VGPRs of the
// 512 lanes (8 per lane, kd-leaf order), so every search evaluates all live
// distances (bit-exact sequential f32 sums) and then proves, from the DFS
// structure, which leaf ANN returns:
//   c* = unique global minimum; for every far step u on c*'s root path,
//   box'(u) < min over near-sibling subtrees before u  ==> c* is visited,
//   hence ANN returns c*.  Otherwise an exact single-lane DFS over the
//   already computed distances decides (rare: ~0.2-2% of searches).
// ============================================================================
struct ScanShared {
    KdTree t;
    float dist[kMaxK];   // live distance per kd-leaf position (also build scratch)
    float rate[kMaxK];   // Single(1/sqrt(previous-pass count)) by kd-leaf position
    int cnta[kMaxK];     // this-pass counts by kd-leaf position
    float wB[8][16];     // per-wave certificate thresholds by LCA depth
    float wmin[8];
    int wcnt[8];
    int wpos[8];
    int wok[8];
    int slow_pos;
    float slow_key;
    int any_nan;                // some centroid of this pass is NaN (yakmo 0/0 means)
    uint8_t nanpos[kMaxK];      // kd-leaf position holds a NaN centroid (fixed for the pass)
};

struct MinRec {
    float v;
    int cnt;
    int pos;
};
__device__ __forceinline__ MinRec min_combine(MinRec a, MinRec b) {
    if (b.v < a.v) return b;
    if (a.v < b.v) return a;
    MinRec r;
    r.v = a.v;
    r.cnt = a.cnt + b.cnt;
    r.pos = min(a.pos, b.pos);
    return r;
}


// wave-wide min of non-negative f32 bit patterns (order-preserving as u32;
// NaN sorts above +inf so it only wins when every value is NaN)
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
    const int id = -1;
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x111, 0xf, 0xf, false));  // row_shr:1
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x112, 0xf, 0xf, false));  // row_shr:2
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x114, 0xf, 0xf, false));  // row_shr:4
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x118, 0xf, 0xf, false));  // row_shr:8
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x142, 0xa, 0xf, false));  // row_bcast:15
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// workgroup barrier that orders LDS only: global stores issued in the search
// loop (cluster ids, live centroid mirror) stay in flight across it
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// One KNNScanReduce pass (encoder.lpr:725-761) for every frame of the batch;
// the host launches it until every frame converged (<= 100 passes).  Frames
// that already converged return immediately.  blockDim = 64 * ceil(K / 512).
template <int D>
__global__ __launch_bounds__(kScanThreads) void scan_pass_kernel(ReduceFrame* __restrict__ frames, int nframes,
                                                                  const float* __restrict__ Xall,
                                                                  float* __restrict__ Call, int* __restrict__ i_scratch,
                                                                  float* __restrict__ f_scratch,
                                                                  const float* __restrict__ rate_tab, double tol,
                                                                  int max_passes, int only_flagged) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    ScanShared& sh = *reinterpret_cast<ScanShared*>(smem);
    const int fi = blockIdx.x;
    if (fi >= nframes) return;
    ReduceFrame* frp = frames + fi;
    if (uniform_int(frp->done)) return;
    if (only_flagged && !uniform_int(frp->generic)) return;  // the batched kernel ran this pass
    const int pass = uniform_int(frp->iters);  // frames advance on their own pass counts
    if (pass >= max_passes) return;
    const int N = uniform_int(frp->N), K = uniform_int(frp->K);
    const int dcol_i = uniform_int(frp->dcol) > 0 ? uniform_int(frp->dcol) : D;
    // best / colCount: a constant power-of-two divisor (an exact multiply) unless the slab is padded
    auto per_col = [dcol_i](float v) { return dcol_i == D ? v / (float)D : v / (float)dcol_i; };
    const float* __restrict__ X = Xall + uniform_i64(frp->x_off);
    float* C = Call + uniform_i64(frp->c_off);
    int* clusters = i_scratch + uniform_i64(frp->n_off);
    int* prev_cnt = i_scratch + uniform_i64(frp->k_off);  // cnts[not Odd(iter)] by centroid id
    float* box0 = f_scratch + uniform_i64(frp->n_off * 3);  // root box per query (yakmo scratch reused)
    int* first = reinterpret_cast<int*>(box0 + N);            // first leaf of ANN's descent per query
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nthreads = blockDim.x, nwaves = nthreads >> 6;
    const bool pow2 = (K & (K - 1)) == 0;
    const int log2K = 31 - __clz(K);

    if (pass == 0)
        for (int k = tid; k < K; k += nthreads) prev_cnt[k] = 1;  // CCntStart (encoder.lpr:717-721)
    if (tid == 0) sh.any_nan = 0;
    __syncthreads();
    build_tree<D>(sh.t, sh.dist, C, K);
    // annBoxDistance(q, bnd_lo, bnd_hi) for every query of this pass
    for (int i = tid; i < N; i += nthreads) {
        const float* qp = X + (int64_t)i * D;
        float box = 0.0f;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const float qd = qp[d];
            if (qd < sh.t.bnd_lo[d]) {
                const float t = fsub(sh.t.bnd_lo[d], qd);
                box = fadd(box, fmul(t, t));
            } else if (qd > sh.t.bnd_hi[d]) {
                const float t = fsub(qd, sh.t.bnd_hi[d]);
                box = fadd(box, fmul(t, t));
            }
        }
        box0[i] = box;
        // the leaf ANN's DFS reaches first: near children only (annkSearch never
        // prunes on the way down); the stale tree fixes it for the whole pass
        int h = 0, s = 0, n = K;
        while (n > 1) {
            const int half = n >> 1;
            if (fsub(qp[sh.t.cd[h]], sh.t.cv[h]) < 0.0f) {
                h = 2 * h + 1;
                n = half;
            } else {
                h = 2 * h + 2;
                s += half;
                n -= half;
            }
        }
        first[i] = s;
    }

    float creg[kScanSlots][D];
    const int p0 = tid * kScanSlots;  // kd-leaf positions [p0, p0+8) live in this lane
#pragma unroll
    for (int s = 0; s < kScanSlots; ++s) {
        const int p = p0 + s;
        if (p < K) {
            const int id = sh.t.pidx[p];
#pragma unroll
            for (int d = 0; d < D; ++d) creg[s][d] = C[(int64_t)id * D + d];
            sh.rate[p] = rate_tab[prev_cnt[id]];  // Single(1/sqrt(cnts[not Odd(iter)]))
            sh.cnta[p] = 1;
            // a centroid is NaN for the whole pass or for none of it: a NaN row
            // stays NaN under c + (x - c) * rate, a finite one stays finite
            bool nn = false;
#pragma unroll
            for (int d = 0; d < D; ++d) nn |= creg[s][d] != creg[s][d];
            sh.nanpos[p] = nn ? 1 : 0;
            if (nn) sh.any_nan = 1;
        } else {
#pragma unroll
            for (int d = 0; d < D; ++d) creg[s][d] = 0.0f;
        }
    }
    // depth of the kd tree: leaves at depth <= maxdepth
    int maxdepth = 0;
    while ((1 << maxdepth) < K) ++maxdepth;
    __syncthreads();

    double err = 0.0;  // thread 0
    int slow_total = 0;
    for (int i = 0; i < N; ++i) {
        const float* qp = X + (int64_t)i * D;
        float q[D];
#pragma unroll
        for (int d = 0; d < D; ++d) q[d] = qp[d];
        const float rootbox = box0[i];
        // ---- phase A: live distances of this lane's 8 kd leaves ----
        float dv[kScanSlots];
#pragma unroll
        for (int s = 0; s < kScanSlots; ++s) dv[s] = 0.0f;
        // ANN leaf distance: dist = dist + (q[d]-p[d])^2 for d = 0..D-1
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const float qd = q[d];
#pragma unroll
            for (int s = 0; s < kScanSlots; ++s) {
                const float t = fsub(qd, creg[s][d]);
                dv[s] = fadd(dv[s], fmul(t, t));
            }
        }
        uint32_t lmin = 0xffffffffu;
#pragma unroll
        for (int s = 0; s < kScanSlots; ++s)
            if (p0 + s < K) lmin = min(lmin, __float_as_uint(dv[s]));
        const uint32_t wmin = wave_min_u32(lmin);
        uint64_t any = 0;
        int wcnt = 0;
        uint64_t masks[kScanSlots];
#pragma unroll
        for (int s = 0; s < kScanSlots; ++s) {
            masks[s] = __ballot((p0 + s < K) && __float_as_uint(dv[s]) == wmin);
            wcnt += __popcll(masks[s]);
            any |= masks[s];
        }
        int wpos = 0x7fffffff;
        if (any) {
            const int l = __ffsll((long long)any) - 1;
            int slot = kScanSlots;
#pragma unroll
            for (int s = kScanSlots - 1; s >= 0; --s)
                if ((masks[s] >> l) & 1ull) slot = s;
            wpos = (wave * 64 + l) * kScanSlots + slot;
        }
        if (lane == 0) {
            sh.wmin[wave] = __uint_as_float(wmin);
            sh.wcnt[wave] = wcnt;
            sh.wpos[wave] = wpos;
        }
        lds_barrier();
        // ---- phase B: certificate that ANN's DFS visits the global minimum ----
        MinRec g;
        g.v = sh.wmin[0];
        g.cnt = sh.wcnt[0];
        g.pos = sh.wpos[0];
        for (int w = 1; w < nwaves; ++w) {
            MinRec o;
            o.v = sh.wmin[w];
            o.cnt = sh.wcnt[w];
            o.pos = sh.wpos[w];
            g = min_combine(g, o);
        }
        // NaN centroids: a NaN leaf reached first becomes ANN's answer (its
        // key NaN fails every later box' < key test, so the DFS ends there);
        // after a real first leaf every NaN leaf is inert (key > NaN is false),
        // so the certificate below may treat NaN distances as +inf
        const int fl = uniform_int(sh.any_nan) ? uniform_int(first[i]) : -1;
        const bool nanfirst = fl >= 0 && sh.nanpos[fl] != 0;
        bool fast = !nanfirst && (g.cnt == 1) && (g.v <= FLT_MAX);
        const int pstar = g.pos;
        if (fast) {
            // lane l < maxdepth evaluates the split node at depth l on c*'s path
            bool far = false;
            float inc = 0.0f;
            if (lane < maxdepth) {
                int h, s, n;
                bool golo;
                if (pow2) {
                    const int sh_ = log2K - lane;
                    h = (1 << lane) - 1 + (pstar >> sh_);
                    s = (pstar >> sh_) << sh_;
                    n = K >> lane;
                    golo = ((pstar >> (sh_ - 1)) & 1) == 0;
                } else {
                    h = 0;
                    s = 0;
                    n = K;
                    for (int l = 0; l < lane && n >= 2; ++l) {
                        const int half = n >> 1;
                        if (pstar < s + half) {
                            h = 2 * h + 1;
                            n = half;
                        } else {
                            h = 2 * h + 2;
                            s += half;
                            n -= half;
                        }
                    }
                    golo = pstar < s + (n >> 1);
                }
                if (n >= 2) {
                    const int cdim = sh.t.cd[h];
                    // q[cdim] straight from the query row: a cross-lane read
                    // here would source lanes >= maxdepth, which are inactive
                    // in this branch (cut dims reach D - 1 = 31 at ChunkSize 16)
                    const float qc = qp[cdim];
                    const float cut = fsub(qc, sh.t.cv[h]);
                    const bool nearlo = cut < 0.0f;
                    if (golo != nearlo) {
                        float bd = nearlo ? fsub(sh.t.lo[h], qc) : fsub(qc, sh.t.hi[h]);
                        if (bd < 0.0f) bd = 0.0f;
                        far = true;
                        inc = fsub(fmul(cut, cut), fmul(bd, bd));
                    }
                }
            }
            const uint64_t farmask = __ballot(far);
            // a NaN box' (a NaN cut value or cell bound: NaN centroids) fails
            // ANN's visit test (box' < max_key) whatever the distances, and
            // fmaxf below would drop it from B: such paths take the exact DFS
            const bool nanbox = __ballot(far && inc != inc) != 0;
            // box' = ((root + inc_a) + inc_b) + ... over far steps, in depth order
            float box = rootbox;
            float boxp = -__builtin_inff();
            for (int l = 0; l < maxdepth; ++l) {
                if ((farmask >> l) & 1ull) {
                    box = fadd(box, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(inc), l)));
                    if (lane == l) boxp = box;
                }
            }
            // B[l] = max box' over far steps at depth >= l (lane l holds B[l])
            float B = -__builtin_inff(), run = -__builtin_inff();
            for (int l = maxdepth - 1; l >= 0; --l) {
                run = fmaxf(run, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(boxp), l)));
                if (lane == l) B = run;
            }
            if (lane < 16) sh.wB[wave][lane] = B;  // per-wave table, read back by LCA depth
            // every leaf x in the near sibling of a far step u at depth l needs
            // d(x) > B[l]; then cur(t_u) > box'(u) at every far step: ANN visits c*
            bool ok = true;
            const int plast = min(p0 + kScanSlots, K) - 1;
            const bool mine = pstar >= p0 && pstar <= plast;
            int lv0 = 0, lv1 = 0;
            if (p0 < K && !mine) {
                lv0 = lca_depth(p0, pstar, K, log2K, pow2);
                lv1 = lca_depth(plast, pstar, K, log2K, pow2);
            }
            if (p0 < K) {
                const float thr0 = sh.wB[wave][lv0 & 15];
                if (!mine && lv0 == lv1) {
                    if ((farmask >> lv0) & 1ull) {
#pragma unroll
                        for (int s2 = 0; s2 < kScanSlots; ++s2)
                            if (p0 + s2 < K && dv[s2] <= thr0) ok = false;
                    }
                } else {
#pragma unroll
                    for (int s2 = 0; s2 < kScanSlots; ++s2) {
                        const int p = p0 + s2;
                        if (p >= K || p == pstar) continue;
                        const int lv = lca_depth(p, pstar, K, log2K, pow2);
                        if (((farmask >> lv) & 1ull) && dv[s2] <= sh.wB[wave][lv]) ok = false;
                    }
                }
            }
            fast = __all(ok) && !nanbox;
        }
        if (lane == 0) sh.wok[wave] = fast ? 1 : 0;
        lds_barrier();
        bool allok = true;
        for (int w = 0; w < nwaves; ++w) allok = allok && (sh.wok[w] != 0);
        int bpos;
        float bkey;
        if (nanfirst) {
            bpos = fl;
            bkey = __builtin_nanf("");
        } else if (allok) {
            bpos = pstar;
            bkey = g.v;
        } else {
            // exact DFS over all live distances (rare)
#pragma unroll
            for (int s = 0; s < kScanSlots; ++s)
                if (p0 + s < K) sh.dist[p0 + s] = dv[s];
            __syncthreads();
            if (tid == 0) scan_exact_dfs<D>(sh.t, sh.dist, q, K, C, sh.slow_pos, sh.slow_key);
            __syncthreads();
            bpos = sh.slow_pos;
            bkey = sh.slow_key;
            ++slow_total;
        }
        // ---- phase C: online update of the chosen centroid (encoder.lpr:735-744) ----
        if (bpos >= 0) {
            const int owner = __builtin_amdgcn_readfirstlane(bpos / kScanSlots);
            const int slot = __builtin_amdgcn_readfirstlane(bpos - owner * kScanSlots);
            const bool me = tid == owner;
            const float rate = sh.rate[bpos];
            const int id = sh.t.pidx[bpos];
            // uniform branch on the slot, lane-select on the owner: the 8xD
            // centroid block stays in VGPRs (no dynamic register indexing)
#pragma unroll
            for (int s = 0; s < kScanSlots; ++s) {
                if (s == slot) {
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        const float o = creg[s][d];
                        const float nv = fadd(o, fmul(fsub(q[d], o), rate));
                        creg[s][d] = me ? nv : o;
                        if (me) C[(int64_t)id * D + d] = nv;  // live mirror for the exact DFS
                    }
                }
            }
            if (me) sh.cnta[bpos] += 1;
            if (tid == 0) {
                clusters[i] = id;
                err += (double)sqrt_rn(per_col(bkey));
            }
        }
    }
    __syncthreads();
    // write back the live centroids and this pass's counts (cnts[Odd(iter)])
#pragma unroll
    for (int s = 0; s < kScanSlots; ++s) {
        const int p = p0 + s;
        if (p < K) {
            const int id = sh.t.pidx[p];
#pragma unroll
            for (int d = 0; d < D; ++d) C[(int64_t)id * D + d] = creg[s][d];
            prev_cnt[id] = sh.cnta[p];
        }
    }
    if (tid == 0) {
        const double prev_err = pass == 0 ? 3.4028234663852886e+38 : frp->err;  // err := MaxSingle
        const double diff = err > prev_err ? err - prev_err : prev_err - err;
        frp->iters = pass + 1;
        frp->slow += slow_total;
        frp->err = err;
        frp->done = (diff <= tol || pass + 1 >= kMaxScanIters) ? 1 : 0;
        frp->generic = 0;
    }
}

// ============================================================================
// KNNFit: brute-force 64-NN equivalent with the reference tie rule.
// Candidate f = 4c + 2neg + rev (encoder.lpr:930-938); neg variants are the
// exact negation of the forward values (IEEE division is sign-symmetric),
// rev variants index the chunk backwards.  Pass 1: e0 = min distance.
// Pass 2: best = smallest f with sqrtf(e_f/CS) - sqrtf(e0/CS) <= eps; if more
// than 64 candidates qualify, ANN's bucket order would matter -> flagged.
// ============================================================================
template <int CS>
__device__ __forceinline__ void knn_chunk_dists(const float (&q)[CS], const float* v, float (&e)[4]) {
    e[0] = e[1] = e[2] = e[3] = 0.0f;
#pragma unroll
    for (int j = 0; j < CS; ++j) {
        const float vf = v[j], vr = v[CS - 1 - j];
        const float t0 = fsub(q[j], vf), t1 = fsub(q[j], vr), t2 = fsub(q[j], -vf), t3 = fsub(q[j], -vr);
        e[0] = fadd(e[0], fmul(t0, t0));
        e[1] = fadd(e[1], fmul(t1, t1));
        e[2] = fadd(e[2], fmul(t2, t2));
        e[3] = fadd(e[3], fmul(t3, t3));
    }
}

// Bound-then-exact: the expanded form |q|^2 + |v|^2 -+ 2 q.v (fma dot
// products; one dot serves a candidate and its negation) is within
// eps_b = (|q|^2 + vmax) 2^-17 of the exact sequential distance (error budget:
// fma dot <= CS u (|q|^2 + |v|^2)/2 x 2, norms <= CS u each, two adds, the
// exact sum <= (CS + 1) u x 2 (|q|^2 + |v|^2): < 90 u for CS <= 16, against
// 128 u).  The exact distances are computed only where the bounds cannot decide:
// pass 1 evaluates a candidate exactly only while its bound is within 2 eps_b of
// the running minimum bound (the exact minimum always is, as the threshold only
// falls); pass 2 only where some variant's bound may reach the acceptance
// threshold, which is monotone in e, so skipped variants cannot qualify.  The
// chosen index and the tie count are those of the all-exact scan.
template <int CS>
__global__ __launch_bounds__(256) void knnfit_kernel(FitFrame* __restrict__ frames, int nframes,
                                                      const float* __restrict__ cand_all, const float* __restrict__ q_all,
                                                      int* __restrict__ out_all, int tiles_per_frame, int tile_r) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* tile = reinterpret_cast<float*>(smem);
    float* vvt = tile + (size_t)tile_r * CS;  // |v|^2 per candidate of the tile
    __shared__ unsigned int s_vmax;
    const int fi = blockIdx.x / tiles_per_frame;
    const int ti = blockIdx.x - fi * tiles_per_frame;
    if (fi >= nframes) return;
    FitFrame* fr = frames + fi;
    const int R = fr->R, N = fr->N;
    const float eps = fr->eps;
    const float* cand = cand_all + fr->cand_off;
    if (ti * 256 >= N) return;  // whole block idle (uniform)
    const int qi = ti * 256 + threadIdx.x;
    const bool active = qi < N;
    float q[CS];
#pragma unroll
    for (int j = 0; j < CS; ++j) q[j] = active ? q_all[fr->q_off + (int64_t)qi * CS + j] : 0.0f;
    // vmax >= |v|^2 over the frame's candidates (nonnegative floats order as their bits)
    if (threadIdx.x == 0) s_vmax = 0u;
    __syncthreads();
    {
        unsigned int m = 0u;
        for (int c = threadIdx.x; c < R; c += 256) {
            float vv = 0.0f;
#pragma unroll
            for (int j = 0; j < CS; ++j) vv = __fmaf_rn(cand[(int64_t)c * CS + j], cand[(int64_t)c * CS + j], vv);
            m = max(m, __float_as_uint(vv * 1.0000153f));  // NaN bits exceed +inf: eb = NaN, nothing is skipped
        }
        atomicMax(&s_vmax, m);
    }
    float qq = 0.0f;
#pragma unroll
    for (int j = 0; j < CS; ++j) qq = __fmaf_rn(q[j], q[j], qq);
    __syncthreads();
    const float eb = (qq + __uint_as_float(s_vmax)) * 7.62939453e-06f;  // 2^-17
    float e0 = __builtin_inff(), mt = __builtin_inff();
    float s0 = 0.0f, ehi = 0.0f;
    int best = -1, cnt = 0;
    for (int pass = 0; pass < 2; ++pass) {
        for (int c0 = 0; c0 < R; c0 += tile_r) {
            const int nr = min(tile_r, R - c0);
            __syncthreads();
            for (int k = threadIdx.x; k < nr * CS; k += 256) tile[k] = cand[(int64_t)c0 * CS + k];
            __syncthreads();
            for (int c = threadIdx.x; c < nr; c += 256) {
                float vv = 0.0f;
#pragma unroll
                for (int j = 0; j < CS; ++j) vv = __fmaf_rn(tile[c * CS + j], tile[c * CS + j], vv);
                vvt[c] = vv;
            }
            __syncthreads();
            for (int c = 0; c < nr; ++c) {
                const float* v = tile + c * CS;
                float df = 0.0f, dr = 0.0f;
#pragma unroll
                for (int j = 0; j < CS; ++j) {
                    df = __fmaf_rn(q[j], v[j], df);
                    dr = __fmaf_rn(q[j], v[CS - 1 - j], dr);
                }
                const float base = qq + vvt[c];
                const float mn = base - 2.0f * fmaxf(fabsf(df), fabsf(dr));  // min over the 4 variants
                if (pass == 0) {
                    mt = fminf(mt, mn);
                    if (!(mn > mt + 2.0f * eb)) {  // (a NaN bound evaluates exactly)
                        float e[4];
                        knn_chunk_dists<CS>(q, v, e);
#pragma unroll
                        for (int k = 0; k < 4; ++k) e0 = (e[k] < e0) ? e[k] : e0;
                    }
                } else if (!(mn - eb > ehi)) {
                    float e[4];
                    knn_chunk_dists<CS>(q, v, e);
                    // f order: 4c+0 fwd, 4c+1 rev, 4c+2 neg fwd, 4c+3 neg rev
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const float s = sqrt_rn(e[k] / (float)CS);
                        const float dlt = s0 > s ? fsub(s0, s) : fsub(s, s0);
                        if (dlt <= eps) {
                            if (best < 0) best = 4 * (c0 + c) + k;
                            ++cnt;
                        }
                    }
                }
            }
        }
        if (pass == 0) {
            s0 = sqrt_rn(e0 / (float)CS);
            // acceptance is monotone in e: e > CS (s0 + eps)^2 (1 + 2^-16) never qualifies
            const float t = s0 + eps;
            ehi = (float)CS * t * t * 1.0000153f;
        }
    }
    if (active) {
        out_all[fr->out_off + qi] = (cnt > 64) ? -1 : best;
        if (cnt > 64) atomicAdd(&fr->overflow, 1);
    }
}

}  // namespace gsc

// ---------------------------------------------------------------------------
// launch wrappers (C linkage for the runtime translation unit)
// ---------------------------------------------------------------------------
using namespace gsc;

extern "C" hipError_t gsc_launch_scan_pass(int D, ReduceFrame* frames, int nframes, int K, const float* X, float* C,
                                           int* is, float* fs, const float* rate_tab, double tol, int max_passes,
                                           int only_flagged, hipStream_t st) {
    const int waves = (K + 64 * kScanSlots - 1) / (64 * kScanSlots);
    dim3 grid(nframes), block(64 * waves);
    const size_t shm = sizeof(ScanShared);
    switch (D) {
    case 8:
        (void)hipFuncSetAttribute((const void*)scan_pass_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
        hipLaunchKernelGGL(scan_pass_kernel<8>, grid, block, shm, st, frames, nframes, X, C, is, fs, rate_tab, tol, max_passes, only_flagged);
        break;
    case 16:
        (void)hipFuncSetAttribute((const void*)scan_pass_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
        hipLaunchKernelGGL(scan_pass_kernel<16>, grid, block, shm, st, frames, nframes, X, C, is, fs, rate_tab, tol, max_passes, only_flagged);
        break;
    case 32:
        (void)hipFuncSetAttribute((const void*)scan_pass_kernel<32>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
        hipLaunchKernelGGL(scan_pass_kernel<32>, grid, block, shm, st, frames, nframes, X, C, is, fs, rate_tab, tol, max_passes, only_flagged);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

extern "C" hipError_t gsc_launch_knnfit(int CS, FitFrame* frames, int nframes, int max_n, int max_r,
                                        const float* cand, const float* q, int* out, hipStream_t st) {
    const int tiles = (max_n + 255) / 256;
    dim3 grid(nframes * tiles), block(256);
    // 72 KB tiles (values + |v|^2): two workgroups per CU
    int tile_r = (72 * 1024) / ((CS + 1) * (int)sizeof(float));
    if (tile_r > max_r) tile_r = max_r;
    if (tile_r < 1) tile_r = 1;
    size_t shm = (size_t)tile_r * (CS + 1) * sizeof(float);
    switch (CS) {
#define KF(CSV)                                                                                                   \
    case CSV:                                                                                                     \
        if (hipError_t e = hipFuncSetAttribute((const void*)knnfit_kernel<CSV>,                                   \
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm))             \
            return e;                                                                                             \
        hipLaunchKernelGGL(knnfit_kernel<CSV>, grid, block, shm, st, frames, nframes, cand, q, out, tiles, tile_r);          \
        break;
        KF(1) KF(2) KF(3) KF(4) KF(5) KF(6) KF(7) KF(8) KF(9) KF(10) KF(11) KF(12) KF(13) KF(14) KF(15) KF(16)
#undef KF
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
