// KNNScanReduce (encoder.lpr:699-765) as a batched, speculative pipeline on
// one CU per frame -- the hot kernel of the SoundChunks encode path.
//
// Reference semantics: per pass, ANN builds a kd-tree over the centroids
// (ann_kdtree_create, encoder.lpr:729) and then, for every point i in order,
// runs an exact k = 1 search on that *stale* tree with the *live* centroids
// (the tree keeps the caller's row pointers; encoder.lpr:733) and moves the
// found centroid towards the point (encoder.lpr:735-744).  Point i+1 sees the
// update of point i, so the chain is sequential.  Only ONE centroid moves per
// point, which is what this kernel exploits.
//
// Layout: the K = 2^LOGK centroids live in VGPRs, 8 consecutive kd-leaf
// positions per lane (K = 4096: 8 waves x 64 lanes x 8 x D floats), so leaf
// position p = (wave*64 + lane)*8 + slot and every kd subtree is an aligned
// block of waves / lanes / slots.
//
// Pipeline, per iteration (batches of kBatch queries):
//   S  (wave 0)   serial commit of the PREVIOUS batch: for each query, check
//                 its speculative answer against the update log (the <= 64
//                 centroids moved since the snapshot its distances were
//                 computed on), then apply the online update to the log.
//   A1 (all)      snapshot distances of the CURRENT batch: every lane computes
//                 its 8 leaf distances (bit-exact sequential f32, no FMA), and
//                 a wave min-tree (DPP) yields per wave: min, tie flag, argmin
//                 position and the min of every sibling subtree on the path
//                 to that argmin.
//   A2 (all)      per query: global argmin c*, the ANN DFS certificate on c*'s
//                 root path (box' of every far step vs the min of the sibling
//                 subtree visited before it), second minimum m2.
//   refresh       owners fold the log into their registers.
// A query whose certificate or log check fails restarts the pipeline at that
// query with a fresh snapshot; if it fails on a fresh snapshot it is resolved
// by the exact single-lane DFS (scan_exact_dfs) over live distances.
//
// Certificate (why c* is ANN's answer): c* is the unique global minimum; ANN
// visits c* iff at every far step u on c*'s root path box'(u) < best-so-far;
// best-so-far there is a minimum over leaves of the near-sibling subtrees of
// far steps at depth <= depth(u).  So "min(sibling subtree at far depth l) >
// max_{far l' >= l} box'(l')" for every far l proves the visit; once visited
// the unique minimum is never replaced.
#include "gsc_tree.h"

namespace gsc {

constexpr int kBatch = 32;  // queries per speculative batch (log window 2*kBatch <= 64)

struct WaveRec {      // A1 output per (wave, query)
    uint32_t minbits; // wave minimum distance (f32 bits; distances are >= 0)
    int tie;          // >= 2 leaves of this wave at the minimum
    int pos;          // first kd-leaf position at the minimum
    uint32_t sib[9];  // sibling-subtree minima on the path to pos:
                      // [b] lane groups of 2^b lanes (b = 0..5),
                      // [6] sibling slot, [7] other slot pair, [8] other slot quad
};

struct QRec {         // A2 output per query
    int valid;
    int cstar;        // kd-leaf position of the certified answer
    int id;           // centroid id (pidx[cstar])
    float g;          // snapshot distance to c*
    float m2;         // snapshot minimum over every other leaf
    float rate;       // Single(1/sqrt(previous-pass count of c*))
    uint32_t farmask; // far steps on c*'s root path, bit = depth
    int pad_;
    float B[12];      // suffix max of box' over far steps (certificate thresholds)
    float o[16];      // c*'s snapshot coordinates
};

struct Scan2Shared {
    KdTree t;
    float dist[kMaxK];  // tree build scratch; live distances for the exact DFS
    float rate[kMaxK];  // Single(1/sqrt(cnts[not Odd(iter)])) by kd-leaf position
    int cnta[kMaxK];    // cnts[Odd(iter)] by kd-leaf position
    float q[2][kBatch][16];
    float qslow[16];
    WaveRec wrec[8][kBatch];
    QRec qrec[2][kBatch];
    int pub_pos[64];
    float pub_c[64][16];
    float lg_c[64][16];  // update log coordinates (wave 0's lane t owns entry t)
    int fail_j, fail_slow;
    int slow_pos;
    float slow_key;
    int any_nan;
    int st_h[16];       // exact-DFS stack (one lane)
    float st_box[16];
};

#ifdef GSC_STAMPS
// diagnostic build: s_memtime per pipeline phase (cdna_hip_programming.md §7)
__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define STAMP(k)                          \
    {                                     \
        const uint64_t t_ = stamp();      \
        acc[k] += t_ - tlast;             \
        tlast = t_;                       \
    }
#else
#define STAMP(k)
#endif

__device__ __forceinline__ uint32_t rl(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ float rlf(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// value of the lane in the other aligned half of the 2^(b+1) lane group
// (valid for group-uniform inputs, which the min-tree guarantees)
template <int B>
__device__ __forceinline__ uint32_t partner(uint32_t v) {
    if constexpr (B == 0) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    if constexpr (B == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    if constexpr (B == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
    if constexpr (B == 3) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
    if constexpr (B == 4) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);                      // xor 16
    return 0u;
}

// ---------------------------------------------------------------------------
// A1: snapshot distances of one query against this wave's 512 leaves.
// ---------------------------------------------------------------------------
template <int D, int LOGK>
__device__ __forceinline__ void a1_query(Scan2Shared& sh, const float (&creg)[8][D], const float* __restrict__ qv,
                                         WaveRec& rec, int wave, int lane) {
    constexpr int K = 1 << LOGK;
    const int p0 = (wave * 64 + lane) * 8;
    float q[D];
#pragma unroll
    for (int d = 0; d < D; ++d) q[d] = qv[d];
    // ANN leaf distance (ANN.dll @0x1800128b0): dist = dist + (q[d]-p[d])^2, d = 0..D-1
    float dv[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) dv[s] = 0.0f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const float t = fsub(q[d], creg[s][d]);
            dv[s] = fadd(dv[s], fmul(t, t));
        }
    }
    uint32_t b[8];
    const bool has = p0 < K;
#pragma unroll
    for (int s = 0; s < 8; ++s) b[s] = has ? __float_as_uint(dv[s]) : 0xFFFFFFFFu;
    const uint32_t m01 = min(b[0], b[1]), m23 = min(b[2], b[3]), m45 = min(b[4], b[5]), m67 = min(b[6], b[7]);
    const uint32_t m03 = min(m01, m23), m47 = min(m45, m67);
    const uint32_t lmin = min(m03, m47);
    int ls = 7, lc = 0;
#pragma unroll
    for (int s = 7; s >= 0; --s) {
        const bool e = b[s] == lmin;
        lc += e ? 1 : 0;
        ls = e ? s : ls;
    }
    // in-lane sibling minima of slot ls: slot ls^1, pair (ls>>1)^1, quad (ls>>2)^1
    const uint32_t pa = (ls & 4) ? ((ls & 2) ? b[6] : b[4]) : ((ls & 2) ? b[2] : b[0]);
    const uint32_t pb = (ls & 4) ? ((ls & 2) ? b[7] : b[5]) : ((ls & 2) ? b[3] : b[1]);
    const uint32_t s0 = (ls & 1) ? pa : pb;
    const uint32_t s1 = (ls & 4) ? ((ls & 2) ? m45 : m67) : ((ls & 2) ? m01 : m23);
    const uint32_t s2 = (ls & 4) ? m03 : m47;
    // wave min-tree: partner group minima are the sibling subtrees on the path
    uint32_t v = lmin;
    const uint32_t sl0 = partner<0>(v);
    v = min(v, sl0);
    const uint32_t sl1 = partner<1>(v);
    v = min(v, sl1);
    const uint32_t sl2 = partner<2>(v);
    v = min(v, sl2);
    const uint32_t sl3 = partner<3>(v);
    v = min(v, sl3);
    const uint32_t sl4 = partner<4>(v);
    v = min(v, sl4);
    const uint32_t vlo = rl(v, 0), vhi = rl(v, 32);
    const uint32_t sl5 = lane < 32 ? vhi : vlo;
    const uint32_t wmin = min(vlo, vhi);
    const uint64_t m = __ballot(lmin == wmin);
    const int L = __ffsll((long long)m) - 1;
    const int tie = (__popcll(m) > 1 || (int)rl((uint32_t)lc, L) > 1) ? 1 : 0;
    const int pos = (wave * 64 + L) * 8 + (int)rl((uint32_t)ls, L);
    const uint32_t r0 = rl(sl0, L), r1 = rl(sl1, L), r2 = rl(sl2, L), r3 = rl(sl3, L), r4 = rl(sl4, L), r5 = rl(sl5, L);
    const uint32_t r6 = rl(s0, L), r7 = rl(s1, L), r8 = rl(s2, L);
    if (lane == 0) {
        rec.minbits = wmin;
        rec.tie = tie;
        rec.pos = pos;
        rec.sib[0] = r0;
        rec.sib[1] = r1;
        rec.sib[2] = r2;
        rec.sib[3] = r3;
        rec.sib[4] = r4;
        rec.sib[5] = r5;
        rec.sib[6] = r6;
        rec.sib[7] = r7;
        rec.sib[8] = r8;
    }
}

// global winner of query jj over the NW wave records (first wave at the minimum)
template <int NW>
__device__ __forceinline__ void winner(const Scan2Shared& sh, int jj, uint32_t& gmin, int& W, int& nmin) {
    gmin = 0xFFFFFFFFu;
    W = 0;
    nmin = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const uint32_t m = sh.wrec[w][jj].minbits;
        if (m < gmin) {
            gmin = m;
            W = w;
            nmin = 1;
        } else if (m == gmin) {
            ++nmin;
        }
    }
}

// ---------------------------------------------------------------------------
// A2: certificate for query jj (one wave, lanes = tree depths).
// ---------------------------------------------------------------------------
template <int D, int LOGK, int NW>
__device__ __forceinline__ void a2_query(Scan2Shared& sh, int jj, int qb, int lane) {
    constexpr int KW = LOGK >= 9 ? LOGK - 9 : 0;  // depths resolved at wave level
    uint32_t gmin;
    int W, nmin;
    winner<NW>(sh, jj, gmin, W, nmin);
    gmin = rfl(gmin);
    W = __builtin_amdgcn_readfirstlane(W);
    nmin = __builtin_amdgcn_readfirstlane(nmin);
    const WaveRec& r = sh.wrec[W][jj];
    const int cstar = __builtin_amdgcn_readfirstlane(r.pos);
    const int tie = (nmin > 1 || r.tie) ? 1 : 0;
    const float* q = sh.q[qb][jj];
    // sibling-subtree minimum at depth l, held by lane l
    uint32_t sib = 0xFFFFFFFFu;
    if (lane < KW) {
        const int sh_ = KW - 1 - lane;  // sibling wave group of W at depth lane
        const int want = (W >> sh_) ^ 1;
#pragma unroll
        for (int w = 0; w < NW; ++w)
            if ((w >> sh_) == want) sib = min(sib, sh.wrec[w][jj].minbits);
    } else if (lane < LOGK) {
        const int idx = lane <= LOGK - 4 ? (LOGK - 4 - lane) : (lane == LOGK - 3 ? 8 : (lane == LOGK - 2 ? 7 : 6));
        sib = r.sib[idx];
    }
    // path evaluation: split node at depth l on c*'s root path (ANNkd_split::ann_search)
    bool far = false;
    float inc = 0.0f;
    if (lane < LOGK) {
        const int h = (1 << lane) - 1 + (cstar >> (LOGK - lane));
        const bool golo = ((cstar >> (LOGK - 1 - lane)) & 1) == 0;
        const int cdim = sh.t.cd[h];
        const float qc = q[cdim];
        const float cut = fsub(qc, sh.t.cv[h]);
        const bool nearlo = cut < 0.0f;
        if (golo != nearlo) {
            float bd = nearlo ? fsub(sh.t.lo[h], qc) : fsub(qc, sh.t.hi[h]);
            if (bd < 0.0f) bd = 0.0f;
            far = true;
            inc = fsub(fmul(cut, cut), fmul(bd, bd));
        }
    }
    const uint64_t farmask = __ballot(far);
    // annBoxDistance(q, enclosing rect) in dimension order
    float box = 0.0f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float qd = q[d];
        if (sh.t.bnd_lo[d] > qd) {
            const float t = fsub(sh.t.bnd_lo[d], qd);
            box = fadd(box, fmul(t, t));
        } else if (qd > sh.t.bnd_hi[d]) {
            const float t = fsub(qd, sh.t.bnd_hi[d]);
            box = fadd(box, fmul(t, t));
        }
    }
    // box' at far steps, accumulated root -> leaf: box' = (cut^2 - bd^2) + box
    float boxp = -__builtin_inff();
    for (int l = 0; l < LOGK; ++l) {
        if ((farmask >> l) & 1ull) {
            box = fadd(box, rlf(inc, l));
            if (lane == l) boxp = box;
        }
    }
    float Bv = -__builtin_inff(), run = -__builtin_inff();
    for (int l = LOGK - 1; l >= 0; --l) {
        run = fmaxf(run, rlf(boxp, l));
        if (lane == l) Bv = run;
    }
    const bool ok = !far || (__uint_as_float(sib) > Bv);
    const bool valid = !tie && __uint_as_float(gmin) <= FLT_MAX && __all(ok);
    // m2: minimum over all sibling subtrees = every leaf except c*
    uint32_t m2 = sib;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) m2 = min(m2, (uint32_t)__shfl_xor((int)m2, o));
    m2 = rl(m2, 0);
    QRec& R = sh.qrec[qb][jj];
    if (lane < LOGK) R.B[lane] = Bv;
    if (lane == 0) {
        R.valid = valid ? 1 : 0;
        R.cstar = cstar;
        R.id = sh.t.pidx[cstar];
        R.g = __uint_as_float(gmin);
        R.m2 = __uint_as_float(m2);
        R.rate = sh.rate[cstar];
        R.farmask = (uint32_t)farmask;
    }
}

// ---------------------------------------------------------------------------
// S: serial commit of a speculated batch (wave 0).  Returns via sh.fail_j.
// Log: lane t holds entry t = (position lg_pos, live coordinates lg_c,
// batch tag lg_bt); every centroid moved since the snapshot of the batch
// being committed is in the log with its live value.
// ---------------------------------------------------------------------------
template <int D, int LOGK>
__device__ __forceinline__ void s_commit(Scan2Shared& sh, int qb, int ps, int pn, bool pfresh, int pit, int lane,
                                         int& lg_pos, int& lg_bt, int* __restrict__ clusters,
                                         double& err) {
    if (lg_pos >= 0 && lg_bt <= pit - 2) lg_pos = -1;  // already folded into the snapshot
    int fj = -1, fslow = 0;
#pragma unroll 1
    for (int jj = 0; jj < pn; ++jj) {
        const QRec& R = sh.qrec[qb][jj];
        const int valid = __builtin_amdgcn_readfirstlane(R.valid);
        if (!valid) {
            fj = jj;
            fslow = (pfresh && jj == 0) ? 1 : 0;
            break;
        }
        const int cstar = __builtin_amdgcn_readfirstlane(R.cstar);
        const float g = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(R.g)));
        const float m2 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(R.m2)));
        const uint32_t farmask = rfl(R.farmask);
        const float* q = sh.q[qb][jj];
        float qd[D];
#pragma unroll
        for (int d = 0; d < D; ++d) qd[d] = q[d];
        float du = 0.0f;
        float* lc = sh.lg_c[lane];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const float t = fsub(qd[d], lc[d]);
            du = fadd(du, fmul(t, t));
        }
        const bool act = lg_pos >= 0;
        const bool isc = act && lg_pos == cstar;
        const uint64_t mc = __ballot(isc);
        const int tc = mc ? __ffsll((long long)mc) - 1 : -1;
        const float gp = tc >= 0 ? rlf(du, tc) : g;
        const bool okc = tc < 0 || gp < m2;
        bool oku = true;
        if (act && !isc) {
            const int lca = __clz(lg_pos ^ cstar) - (32 - LOGK);
            const bool farl = (farmask >> lca) & 1u;
            oku = du > gp && (!farl || du > R.B[lca]);
        }
        if (!(okc && __all(oku))) {
            fj = jj;
            fslow = (pfresh && jj == 0) ? 1 : 0;
            break;
        }
        // online update of c* (encoder.lpr:735-740), f32: c += (x - c) * rate
        const float rate = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(R.rate)));
        const int e = tc >= 0 ? tc : __ffsll((long long)__ballot(lg_pos < 0)) - 1;
        if (lane == e) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const float o = tc >= 0 ? lc[d] : R.o[d];
                lc[d] = fadd(o, fmul(fsub(qd[d], o), rate));
            }
            lg_pos = cstar;
            lg_bt = pit;
        }
        if (lane == 0) {
            sh.cnta[cstar] += 1;
            clusters[ps + jj] = R.id;
            err += (double)__fsqrt_rn(gp / (float)D);  // encoder.lpr:743
        }
    }
    if (fslow) {
        if (lane < D) sh.qslow[lane] = sh.q[qb][fj][lane];
    }
    if (lane == 0) {
        sh.fail_j = fj;
        sh.fail_slow = fslow;
    }
}

// Exact ANN ann_search (k = 1, eps = 0; annkSearch @0x1800124b0) over the
// stale tree with the live leaf distances in sh.dist -- one lane, stack in
// LDS.  No NaN distances reach this kernel (those passes run the generic
// kernel), so leaf early exits cannot change a result.
template <int D, int LOGK>
__device__ __forceinline__ void dfs_exact(Scan2Shared& sh, int& out_pos, float& out_key) {
    constexpr int K = 1 << LOGK;
    const float* q = sh.qslow;
    float cur_box = 0.0f;
    for (int d = 0; d < D; ++d) {  // annBoxDistance
        const float qd = q[d];
        if (sh.t.bnd_lo[d] > qd) {
            const float t = fsub(sh.t.bnd_lo[d], qd);
            cur_box = fadd(cur_box, fmul(t, t));
        } else if (qd > sh.t.bnd_hi[d]) {
            const float t = fsub(qd, sh.t.bnd_hi[d]);
            cur_box = fadd(cur_box, fmul(t, t));
        }
    }
    int h = 0, sp = 0, best = -1;
    float key = FLT_MAX;
    for (;;) {
        if (h >= K - 1) {
            // ANNkd_leaf::ann_search: insert iff the list is empty or key > dist
            const int p = h - (K - 1);
            const float dd = sh.dist[p];
            if (best < 0 || key > dd) {
                key = dd;
                best = p;
            }
            // unwind: the far child is visited iff box' < max_key
            bool found = false;
            while (sp > 0) {
                --sp;
                if (sh.st_box[sp] < key) {
                    h = sh.st_h[sp];
                    cur_box = sh.st_box[sp];
                    found = true;
                    break;
                }
            }
            if (!found) break;
            continue;
        }
        const int cdim = sh.t.cd[h];
        const float qc = q[cdim];
        const float cut = fsub(qc, sh.t.cv[h]);
        float bd;
        int nearh, farh;
        if (cut < 0.0f) {
            bd = fsub(sh.t.lo[h], qc);
            nearh = 2 * h + 1;
            farh = 2 * h + 2;
        } else {
            bd = fsub(qc, sh.t.hi[h]);
            nearh = 2 * h + 2;
            farh = 2 * h + 1;
        }
        if (bd < 0.0f) bd = 0.0f;
        sh.st_box[sp] = fadd(cur_box, fsub(fmul(cut, cut), fmul(bd, bd)));
        sh.st_h[sp] = farh;
        ++sp;
        h = nearh;
    }
    out_pos = best;
    out_key = key;
}

// fold published log entries into the owners' registers
template <int D>
__device__ __forceinline__ void refresh(Scan2Shared& sh, float (&creg)[8][D], int wave, int lane) {
    const int pp = sh.pub_pos[lane];
    uint64_t m = __ballot(pp >= 0 && (pp >> 9) == wave);
    while (m) {
        const int e = __ffsll((long long)m) - 1;
        m &= m - 1;
        const int p = __builtin_amdgcn_readlane(pp, e);
        const int owner = (p >> 3) & 63, slot = p & 7;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            if (s == slot) {
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const float v = sh.pub_c[e][d];
                    creg[s][d] = lane == owner ? v : creg[s][d];
                }
            }
        }
    }
}

template <int D, int LOGK>
__global__ __launch_bounds__(512) void scan_batch_kernel(ReduceFrame* __restrict__ frames, int nframes,
                                                         const float* __restrict__ Xall, float* __restrict__ Call,
                                                         int* __restrict__ i_scratch, const float* __restrict__ rate_tab,
                                                         double tol, int pass) {
    constexpr int K = 1 << LOGK;
    constexpr int NW = K >= 512 ? K / 512 : 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Scan2Shared& sh = *reinterpret_cast<Scan2Shared*>(smem);
    const int fi = blockIdx.x;
    if (fi >= nframes) return;
    ReduceFrame* frp = frames + fi;
    if (uniform_int(frp->done)) return;
    const int N = uniform_int(frp->N);
    const float* __restrict__ X = uniform_ptr(Xall + frp->x_off);
    float* C = uniform_ptr(Call + frp->c_off);
    int* clusters = uniform_ptr(i_scratch + frp->n_off);
    int* prev_cnt = uniform_ptr(i_scratch + frp->k_off);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    if (pass == 0)
        for (int k = tid; k < K; k += blockDim.x) prev_cnt[k] = 1;  // CCntStart (encoder.lpr:717-721)
    if (tid == 0) sh.any_nan = 0;
    __syncthreads();
    build_tree<D>(sh.t, sh.dist, C, K);

    float creg[8][D];
    const int p0 = tid * 8;
    bool nan_here = false;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const int p = p0 + s;
        if (p < K) {
            const int id = sh.t.pidx[p];
#pragma unroll
            for (int d = 0; d < D; ++d) {
                creg[s][d] = C[(int64_t)id * D + d];
                nan_here |= creg[s][d] != creg[s][d];
            }
            sh.rate[p] = rate_tab[prev_cnt[id]];
            sh.cnta[p] = 1;
        } else {
#pragma unroll
            for (int d = 0; d < D; ++d) creg[s][d] = 0.0f;
        }
    }
    if (nan_here) sh.any_nan = 1;
    // first batch's queries
    const int n0 = min(kBatch, N);
    for (int k = tid; k < n0 * D; k += blockDim.x) sh.q[0][k / D][k % D] = X[k];
    __syncthreads();
    if (uniform_int(sh.any_nan)) {
        // NaN centroids (yakmo 0/0 means) make ANN's early exits order dependent:
        // this pass runs in the generic kernel (gsc_kernels.hip)
        if (tid == 0) frp->generic = 1;
        return;
    }

    // wave-0 state: update log + residual
    int lg_pos = -1, lg_bt = 0;
    double err = 0.0;
    int slow_total = 0, restarts = 0;

#ifdef GSC_STAMPS
    uint64_t acc[6] = {0, 0, 0, 0, 0, 0};
    uint64_t tlast = stamp();
#endif
    int cur_s = 0, cur_n = n0, cbuf = 0;
    bool cur_fresh = true;
    int pend_s = 0, pend_n = 0, pbuf = 1, pit = 0;
    bool pend_fresh = false;
    for (int it = 0;; ++it) {
        // ---- part 1: S(pending) on wave 0, A1(current) on every wave
        if (wave == 0) {
            if (pend_n > 0)
                s_commit<D, LOGK>(sh, pbuf, pend_s, pend_n, pend_fresh, pit, lane, lg_pos, lg_bt, clusters, err);
            else if (lane == 0) {
                sh.fail_j = -1;
                sh.fail_slow = 0;
            }
        }
        STAMP(0)
#pragma unroll 1
        for (int jj = 0; jj < cur_n; ++jj) a1_query<D, LOGK>(sh, creg, sh.q[cbuf][jj], sh.wrec[wave][jj], wave, lane);
        STAMP(1)
        __syncthreads();
        STAMP(2)
        // ---- part 2
        const int fj = uniform_int(sh.fail_j), fslow = uniform_int(sh.fail_slow);
        int next_s;
        bool next_fresh;
        if (fj >= 0) {
            next_s = pend_s + fj + (fslow ? 1 : 0);
            next_fresh = true;
            ++restarts;
        } else {
            next_s = cur_s + cur_n;
            next_fresh = false;
            if (cur_n > 0) {
                // c*'s snapshot coordinates, written by the wave that owns c*
                uint64_t won = 0;
                {
                    uint32_t gm;
                    int W = 0, nm;
                    if (lane < cur_n) winner<NW>(sh, lane, gm, W, nm);
                    won = __ballot(lane < cur_n && W == wave);
                }
                while (won) {
                    const int jj = __ffsll((long long)won) - 1;
                    won &= won - 1;
                    const int p = sh.wrec[wave][jj].pos;
                    const int owner = (p >> 3) & 63, slot = p & 7;
#pragma unroll
                    for (int s = 0; s < 8; ++s)
                        if (s == slot && lane == owner) {
#pragma unroll
                            for (int d = 0; d < D; ++d) sh.qrec[cbuf][jj].o[d] = creg[s][d];
                        }
                }
#pragma unroll 1
                for (int jj = wave; jj < cur_n; jj += NW) a2_query<D, LOGK, NW>(sh, jj, cbuf, lane);
            }
        }
        STAMP(3)
        const int nbuf = cbuf ^ 1;  // the pending batch's buffer (S is done with it)
        const int next_n = max(0, min(kBatch, N - next_s));
        for (int k = tid; k < next_n * D; k += blockDim.x)
            sh.q[nbuf][k / D][k % D] = X[(int64_t)next_s * D + k];
        if (wave == 0) {
            sh.pub_pos[lane] = lg_pos;
            if (lg_pos >= 0) {
#pragma unroll
                for (int d = 0; d < D; ++d) sh.pub_c[lane][d] = sh.lg_c[lane][d];
            }
        }
        __syncthreads();
        STAMP(4)
        // ---- part 3: fold the log into the registers
        refresh<D>(sh, creg, wave, lane);
        if (fj >= 0 && wave == 0) lg_pos = -1;  // everything is in the registers now
        if (fslow) {
            // genuine certificate failure on a fresh snapshot: exact ANN DFS
            const int j = pend_s + fj;
            float dv[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) dv[s] = 0.0f;
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const float qd = sh.qslow[d];
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    const float t = fsub(qd, creg[s][d]);
                    dv[s] = fadd(dv[s], fmul(t, t));
                }
            }
#pragma unroll
            for (int s = 0; s < 8; ++s)
                if (p0 + s < K) sh.dist[p0 + s] = dv[s];
            __syncthreads();
            if (tid == 0) dfs_exact<D, LOGK>(sh, sh.slow_pos, sh.slow_key);
            __syncthreads();
            const int bpos = uniform_int(sh.slow_pos);
            if (bpos >= 0) {
                // owner publishes c's coordinates; tid 0 moves it (encoder.lpr:735-744)
                // and the move is folded in through the refresh path
                const int owner = bpos >> 3, slot = bpos & 7;
#pragma unroll
                for (int s = 0; s < 8; ++s)
                    if (s == slot && tid == owner) {
#pragma unroll
                        for (int d = 0; d < D; ++d) sh.pub_c[0][d] = creg[s][d];
                    }
                if (tid < 64) sh.pub_pos[tid] = tid == 0 ? bpos : -1;
                __syncthreads();
                if (tid == 0) {
                    const float key = sh.slow_key;
                    const float rate = sh.rate[bpos];
                    for (int d = 0; d < D; ++d) {
                        const float o = sh.pub_c[0][d];
                        sh.pub_c[0][d] = fadd(o, fmul(fsub(sh.qslow[d], o), rate));
                    }
                    sh.cnta[bpos] += 1;
                    clusters[j] = sh.t.pidx[bpos];
                    err += (double)__fsqrt_rn(key / (float)D);
                }
                __syncthreads();
                refresh<D>(sh, creg, wave, lane);
            }
            ++slow_total;
            __syncthreads();
        }
        STAMP(5)
        if (fj >= 0) {
            pend_n = 0;
        } else {
            pend_s = cur_s;
            pend_n = cur_n;
            pbuf = cbuf;
            pend_fresh = cur_fresh;
            pit = it;
        }
        cur_s = next_s;
        cur_n = next_n;
        cbuf = nbuf;
        cur_fresh = next_fresh;
        if (cur_n == 0 && pend_n == 0) {
            if (tid == 0) frp->loop_iters = it + 1;
            break;
        }
        if (it > 4 * N + 64) {  // progress guard: every query commits within 3 iterations
            if (tid == 0) frp->loop_iters = -1;
            break;
        }
    }
    // write back the live centroids and this pass's counts (cnts[Odd(iter)])
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const int p = p0 + s;
        if (p < K) {
            const int id = sh.t.pidx[p];
#pragma unroll
            for (int d = 0; d < D; ++d) C[(int64_t)id * D + d] = creg[s][d];
            prev_cnt[id] = sh.cnta[p];
        }
    }
#ifdef GSC_STAMPS
    if (lane == 0 && wave < 2)
        for (int k = 0; k < 6; ++k) frp->stamps[wave * 6 + k] += acc[k];
#endif
    if (tid == 0) {
        const double prev_err = pass == 0 ? 3.4028234663852886e+38 : frp->err;  // err := MaxSingle
        const double diff = err > prev_err ? err - prev_err : prev_err - err;
        frp->iters = pass + 1;
        frp->slow += slow_total;
        frp->restarts += restarts;
        frp->err = err;
        frp->done = (diff <= tol || pass + 1 >= kMaxScanIters || frp->loop_iters < 0) ? 1 : 0;
    }
}

}  // namespace gsc

using namespace gsc;

// One batched KNNScanReduce pass for every frame (K = 2^logk, 256..4096,
// D = 8 or 16).  Returns hipErrorInvalidValue for shapes it does not cover.
extern "C" hipError_t gsc_launch_scan_batch(int D, int logk, ReduceFrame* frames, int nframes, const float* X,
                                            float* C, int* is, const float* rate_tab, double tol, int pass,
                                            hipStream_t st) {
    const int K = 1 << logk;
    const int threads = 64 * (K >= 512 ? K / 512 : 1);
    const size_t shm = sizeof(Scan2Shared);
#define SB(DV, LK)                                                                                                     \
    if (D == DV && logk == LK) {                                                                                       \
        (void)hipFuncSetAttribute((const void*)scan_batch_kernel<DV, LK>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  (int)shm);                                                                           \
        hipLaunchKernelGGL((scan_batch_kernel<DV, LK>), dim3(nframes), dim3(threads), shm, st, frames, nframes, X, C,   \
                           is, rate_tab, tol, pass);                                                                   \
        return hipGetLastError();                                                                                      \
    }
    SB(8, 8) SB(8, 9) SB(8, 10) SB(8, 11) SB(8, 12)
    SB(16, 8) SB(16, 9) SB(16, 10) SB(16, 11) SB(16, 12)
#undef SB
    return hipErrorInvalidValue;
}

extern "C" size_t gsc_scan_batch_shared_bytes(void) { return sizeof(Scan2Shared); }
