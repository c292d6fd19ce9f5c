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
// Pipeline, per iteration (batches of kBatch queries; "current" = the batch
// whose distances are computed now, "pending" = the previous batch, whose
// speculative answers are committed now):
//   part 1  A1 (all waves): snapshot distances of the current batch: each lane
//           computes its 8 leaf distances (bit-exact sequential f32, no FMA);
//           a wave min-tree (DPP) gives per wave the minimum, a tie flag, the
//           argmin position and the minimum of every sibling subtree on the
//           path to it.  Wave 0 first chains the pending batch's online
//           updates (c += (x - c) * rate per query, in order per centroid).
//   part 2  V (all waves): every pending query is checked against every
//           centroid moved since its snapshot (the update log + the earlier
//           queries of its batch), with live coordinates.
//           A2 (all waves, 4 queries per wave): ANN DFS certificate of the
//           current batch: global argmin c*, box' of every far step on c*'s
//           root path against the minimum of the sibling subtree visited
//           before it, second minimum m2.
//   part 3  commit the valid prefix of the pending batch (clusters, counts,
//           residual in order, update log), choose the next batch.
//   part 4  owners fold the log into their registers.
// A query that fails restarts the pipeline at that query on a fresh snapshot;
// if it fails on a fresh snapshot it is resolved by the exact single-lane DFS
// (dfs_exact) over live distances.
//
// Certificate (why c* is ANN's answer): c* is the unique global minimum; ANN
// visits c* iff at every far step u on c*'s root path box'(u) < best-so-far;
// best-so-far there is a minimum over leaves of the near-sibling subtrees of
// far steps at depth <= depth(u).  So "min(sibling subtree at far depth l) >
// max_{far l' >= l} box'(l')" for every far l proves the visit; once visited
// the unique minimum is never replaced.  A centroid u moved after the
// snapshot keeps the proof iff its live distance d_u > d(c*) and, when its
// LCA with c* is a far step, d_u > B[lca]; a moved c* needs d(c*) < m2.
#include "gsc_tree.h"

namespace gsc {

constexpr int kBatch = 32;         // queries per speculative batch (log window 2*kBatch <= 64)
constexpr int kVer = 64 + kBatch;  // centroid versions seen by a pending batch
constexpr int kRow = 20;           // coordinate row stride of lane-indexed LDS rows (80 B: no b128 bank conflicts)

// float minimum on f32 bit patterns (A1 values may be negative: the batch
// queries' bounds are |c|^2 - 2 q.c; exact distances are >= +0, where this
// equals the unsigned order).  fminf returns one operand bit for bit: no NaN
// reaches it, and neither an fma chain started at |c|^2 >= +0 nor an exact
// distance ever yields -0.
__device__ __forceinline__ uint32_t fminb(uint32_t a, uint32_t b) {
    return __float_as_uint(fminf(__uint_as_float(a), __uint_as_float(b)));
}
constexpr uint32_t kInfBits = 0x7F800000u;  // +inf: empty leaf / no value
// f32 bits <-> signed-int order key (an involution): the cross-lane min-tree
// runs on integer keys, so no DPP result needs an IEEE canonicalisation
__device__ __forceinline__ int ordkey(uint32_t b) { return (int)(b ^ ((uint32_t)((int32_t)b >> 31) >> 1)); }
__device__ __forceinline__ uint32_t keybits(int k) { return (uint32_t)ordkey((uint32_t)k); }

struct WaveRec {      // A1 output per (wave, query): raw values of the argmin lane L;
                      // the winner's path minima are derived in A2 (rec_* below)
    uint32_t minbits; // wave minimum distance (f32 bits; distances are >= 0)
    int lanebits;     // L | 256 if another lane of the wave also holds the minimum
    uint32_t sl[6];   // lane L's sibling lane-group minima, groups of 2^b lanes (b = 0..5), as order keys
    uint32_t b[8];    // lane L's 8 leaf distances (slots = kd leaves 8L .. 8L+7 of the wave)
};

// first slot of lane L at the wave minimum, and whether another slot ties it
__device__ __forceinline__ int rec_slot(const WaveRec& r, bool* tie2) {
    int ls = 7, lc = 0;
#pragma unroll
    for (int s = 7; s >= 0; --s) {
        const bool e = r.b[s] == r.minbits;
        lc += e ? 1 : 0;
        ls = e ? s : ls;
    }
    *tie2 = lc > 1 || (r.lanebits >> 8) != 0;
    return ls;
}

// sibling-subtree minimum on the path to slot ls: lane groups (idx 0..5),
// sibling slot (6), other slot pair of the quad (7), other quad (8)
__device__ __forceinline__ uint32_t rec_sib(const WaveRec& r, int ls, int idx) {
    if (idx < 6) return keybits((int)r.sl[idx]);
    if (idx == 6) return r.b[ls ^ 1];
    if (idx == 7) {
        const int pb = (ls & 4) | ((ls & 2) ^ 2);
        return fminb(r.b[pb], r.b[pb + 1]);
    }
    const int qb = (ls & 4) ^ 4;
    return fminb(fminb(r.b[qb], r.b[qb + 1]), fminb(r.b[qb + 2], r.b[qb + 3]));
}

struct QRec {         // A2 output per query
    int valid;
    int cstar;        // kd-leaf position of the certified answer
    int id;           // centroid id (pidx[cstar])
    float g;          // snapshot distance to c*
    float m2;         // snapshot minimum over every other leaf
    float rate;       // Single(1/sqrt(previous-pass count of c*))
    uint32_t farmask; // far steps on c*'s root path, bit = depth
    int pad_;
    float B[16];      // suffix max of box' over far steps (certificate thresholds)
    float o[16];      // c*'s snapshot coordinates
};

struct Scan2Shared {
    KdTree t;
    float dist[kMaxK];  // tree build scratch; live distances for the exact DFS
    float rate[kMaxK];  // Single(1/sqrt(cnts[not Odd(iter)])) by kd-leaf position
    float dfs_inc[kMaxK];  // exact DFS: per split node box' increment, sign = near child hi
    alignas(16) float q[2][kBatch][16];
    alignas(16) float qm[2][kBatch][16];  // -2 q (exact), the A1 dot-product operand
    float cnmax[8];
    int fxl[kBatch];   // queries of the current batch re-certified exactly    // per wave: upper bound of |c|^2 over its live centroids (monotone within a pass)
    alignas(16) float qslow[16];       // the query resolved on its own after a failed commit
    WaveRec wrec[8][kBatch + 1];  // column kBatch: the solo query
    alignas(16) QRec qrec[2][kBatch];
    QRec qsolo;
    // update log: entry e = wave-0 lane e (position in a VGPR, coordinates here)
    alignas(16) float lg_c[64][kRow];
    int pub_pos[64];       // log entries to fold into the registers (position, -1 = none)
    alignas(16) float solo_c[kRow];    // coordinates of the solo query's centroid
    double err_out;
    // commit of the pending batch: versions 0..63 = log entries, 64+j = after query j
    int vpos[kVer];
    int vfrom[kVer];   // first query that sees the version
    int vto[kVer];     // last query that sees it
    alignas(16) float newc[kBatch][kRow];
    float gp[kBatch];  // live d(q_j, c*_j)
    int inval[kBatch];
    int nxt[kBatch];   // next query of the batch with the same c* (kBatch = none)
    int ient[kBatch];  // log entry holding c*_j when the commit starts (-1 = none)
    int freel[64];     // commit: free log entries, in lane order
    int asg[64];       // commit: log entry -> centroid position it now holds
    int slow_pos;
    float slow_key;
    int any_nan;
    int pass_done;     // end of pass: the frame converged (or hands the next pass over)
    int st_h[16];      // exact-DFS stack (one lane)
    float st_box[16];
    uint32_t wkey[2][8];  // parallel exact DFS: per-wave next-improvement keys
    alignas(16) float a2s[8][64];     // A2 scratch per wave: box terms by dimension, box' increments by depth
    alignas(16) float a2i[8][64];
};
static_assert(sizeof(Scan2Shared) <= 160 * 1024, "LDS budget (160 KB per CU)");
static_assert(kRow >= 16 + 1, "log rows carry |c|^2 in their last float");

#ifdef GSC_STAMPS
// diagnostic build: s_memtime per pipeline phase (cdna_hip_programming.md §7)
__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define STAMP(k)                     \
    {                                \
        const uint64_t t_ = stamp(); \
        acc[k] += t_ - tlast;        \
        tlast = t_;                  \
    }
#else
#define STAMP(k)
#endif

// value of the lane in the other aligned half of the 2^(b+1) lane group
// (valid for group-uniform inputs, which the reductions below guarantee)
template <int B>
__device__ __forceinline__ uint32_t partner(uint32_t v) {
    // every lane has a source lane in these patterns: no "old" value needed
    if constexpr (B == 0) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
    if constexpr (B == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
    if constexpr (B == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true);  // row_half_mirror
    if constexpr (B == 3) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true);  // row_mirror
    if constexpr (B == 4) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);                      // xor 16
    return 0u;
}
__device__ __forceinline__ uint32_t min16(uint32_t v) {  // min over each aligned 16-lane row
    v = min(v, partner<0>(v));
    v = min(v, partner<1>(v));
    v = min(v, partner<2>(v));
    return min(v, partner<3>(v));
}
__device__ __forceinline__ uint32_t fmin16(uint32_t v) {  // float min over each aligned 16-lane row
    v = fminb(v, partner<0>(v));
    v = fminb(v, partner<1>(v));
    v = fminb(v, partner<2>(v));
    return fminb(v, partner<3>(v));
}
__device__ __forceinline__ uint32_t sum16(uint32_t v) {
    v += partner<0>(v);
    v += partner<1>(v);
    v += partner<2>(v);
    return v + partner<3>(v);
}

__device__ __forceinline__ int wave_of_lane() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// orders this wave's LDS accesses across lanes (lane-to-lane hand-off
// through LDS inside one wave: without it the compiler may reorder them)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// workgroup barrier that orders LDS only: the loop's global traffic (cluster
// ids, count atomics, query prefetch) stays in flight across it
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// sequential f32 squared distance (ANN leaf order d = 0..D-1)
template <int D>
__device__ __forceinline__ float seqdist(const float* __restrict__ a, const float* __restrict__ b) {
    float s = 0.0f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float t = fsub(a[d], b[d]);
        s = fadd(s, fmul(t, t));
    }
    return s;
}

// ---------------------------------------------------------------------------
// A1: snapshot distances of one query against this wave's 512 leaves.
// ---------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ void a1_dist(const float (&creg)[8][D], const float* __restrict__ qv, float (&dv)[8]) {
    // ANN leaf distance (ANN.dll @0x1800128b0): dist = dist + (q[d]-p[d])^2, d = 0..D-1
#pragma unroll
    for (int s = 0; s < 8; ++s) dv[s] = 0.0f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float qd = qv[d];
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const float t = fsub(qd, creg[s][d]);
            dv[s] = fadd(dv[s], fmul(t, t));
        }
    }
}

// wave min-tree over the lanes' 8 leaf distances -> the query's WaveRec
struct A1Tree {
    uint32_t b[8];  // this lane's leaf values (f32 bits)
    uint32_t lmin;
    int sl[6];      // partner lane-group minima (order keys)
    uint64_t m;     // lanes at the wave minimum
};

template <int LOGK>
__device__ __forceinline__ A1Tree a1_tree(const float (&dv)[8], int wave, int lane) {
    constexpr int K = 1 << LOGK;
    const int p0 = (wave * 64 + lane) * 8;
    A1Tree t;
    const bool has = LOGK >= 9 || p0 < K;  // K >= 512: every lane holds 8 leaves
#pragma unroll
    for (int s = 0; s < 8; ++s) t.b[s] = has ? __float_as_uint(dv[s]) : kInfBits;
    const uint32_t m01 = fminb(t.b[0], t.b[1]), m23 = fminb(t.b[2], t.b[3]), m45 = fminb(t.b[4], t.b[5]),
                   m67 = fminb(t.b[6], t.b[7]);
    t.lmin = fminb(fminb(m01, m23), fminb(m45, m67));
    // wave min-tree on order keys: partner group minima are the sibling subtrees on the path
    const int key = ordkey(t.lmin);
    int v = key;
    t.sl[0] = (int)partner<0>((uint32_t)v);
    v = min(v, t.sl[0]);
    t.sl[1] = (int)partner<1>((uint32_t)v);
    v = min(v, t.sl[1]);
    t.sl[2] = (int)partner<2>((uint32_t)v);
    v = min(v, t.sl[2]);
    t.sl[3] = (int)partner<3>((uint32_t)v);
    v = min(v, t.sl[3]);
    // the two widest levels with the gfx950 row / half swaps: p[0] is this
    // lane's copy of the lower row (half), p[1] of the upper one
    const auto p16 = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
    t.sl[4] = (int)((lane & 16) ? p16[0] : p16[1]);
    v = min((int)p16[0], (int)p16[1]);
    const auto p32 = __builtin_amdgcn_permlane32_swap((uint32_t)v, (uint32_t)v, false, false);
    t.sl[5] = (int)((lane & 32) ? p32[0] : p32[1]);
    const int wmin = min((int)p32[0], (int)p32[1]);
    t.m = __ballot(key == wmin);
    return t;
}

__device__ __forceinline__ void a1_store(const A1Tree& t, WaveRec& rec, int lane) {
    const int L = __ffsll((long long)t.m) - 1;
    if (lane == L) {
        rec.minbits = t.lmin;
        rec.lanebits = L | (__popcll(t.m) > 1 ? 256 : 0);
#pragma unroll
        for (int i = 0; i < 6; ++i) rec.sl[i] = (uint32_t)t.sl[i];
#pragma unroll
        for (int s = 0; s < 8; ++s) rec.b[s] = t.b[s];
    }
}

template <int LOGK>
__device__ __forceinline__ void a1_reduce(const float (&dv)[8], WaveRec& rec, int wave, int lane) {
    a1_store(a1_tree<LOGK>(dv, wave, lane), rec, lane);
}

// two queries: both DPP chains are computed before either record store, so
// their latencies overlap
template <int LOGK>
__device__ __forceinline__ void a1_reduce2(const float (&dv0)[8], const float (&dv1)[8], WaveRec& rec0, WaveRec& rec1,
                                           int wave, int lane) {
    const A1Tree t0 = a1_tree<LOGK>(dv0, wave, lane);
    const A1Tree t1 = a1_tree<LOGK>(dv1, wave, lane);
    a1_store(t0, rec0, lane);
    a1_store(t1, rec1, lane);
}

template <int D, int LOGK>
__device__ __forceinline__ void a1_query(const float (&creg)[8][D], const float* __restrict__ qv, WaveRec& rec,
                                         int wave, int lane) {
    float dv[8];
    a1_dist<D>(creg, qv, dv);
    a1_reduce<LOGK>(dv, rec, wave, lane);
}

// ---------------------------------------------------------------------------
// A1 of the batch queries: expanded-form distance bounds instead of the exact
// sums.  A1 keeps s~ = |c|^2 + sum_d fma(-2 q_d, c_d, .) per leaf (16 VALU ops
// instead of 48; the wave min-tree runs in float order); A2 adds |q|^2 once.
// d~ = fl(|q|^2 + s~) differs from the reference's sequential f32 distance d
// (ANN.dll @0x1800128b0) by at most eps(q) = (|q|^2 + M) * 2^-17, with
// M >= |c|^2 over the live centroids: the 16 fma roundings are <= 32u(|c|^2 +
// |q|^2) (every partial sum is within 2(|c|^2 + |q|^2) by Cauchy-Schwarz), the
// two norms <= 16u each, the final add <= 2u, the reference's own sum <= 18u d
// <= 36u(|c|^2 + |q|^2); u = 2^-24, total < 104u against the 128u used.  A2
// certifies only with that margin; what it cannot decide is re-run exactly on
// the same snapshot (fixup in part 2).  The committed distance g is always
// recomputed exactly from c*'s coordinates (vp_end).
// ---------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ void a1_dist_x2(const float (&creg)[8][D], const float (&cn)[8], const float* __restrict__ qm0,
                                           const float* __restrict__ qm1, float (&dv0)[8], float (&dv1)[8]) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        dv0[s] = cn[s];
        dv1[s] = cn[s];
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float m0 = qm0[d], m1 = qm1[d];
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            dv0[s] = __builtin_fmaf(m0, creg[s][d], dv0[s]);
            dv1[s] = __builtin_fmaf(m1, creg[s][d], dv1[s]);
        }
    }
}

template <int D>
__device__ __forceinline__ float norm2_x(const float* __restrict__ v) {  // |v|^2, any order (bounds only)
    float n = 0.0f;
#pragma unroll
    for (int d = 0; d < D; ++d) n = __builtin_fmaf(v[d], v[d], n);
    return n;
}

// max over the wave of a non-negative float (bit order = value order)
__device__ __forceinline__ float wave_max_nonneg(float x) {
    uint32_t k = __float_as_uint(x);
    k = max(k, partner<0>(k));
    k = max(k, partner<1>(k));
    k = max(k, partner<2>(k));
    k = max(k, partner<3>(k));
    k = max(k, partner<4>(k));
    k = max((uint32_t)__builtin_amdgcn_readlane((int)k, 0), (uint32_t)__builtin_amdgcn_readlane((int)k, 32));
    return __uint_as_float(k);
}

__device__ __forceinline__ float fsum16(float v) {  // sum over each aligned 16-lane row, uniform result
    v = fadd(v, __uint_as_float(partner<0>(__float_as_uint(v))));
    v = fadd(v, __uint_as_float(partner<1>(__float_as_uint(v))));
    v = fadd(v, __uint_as_float(partner<2>(__float_as_uint(v))));
    return fadd(v, __uint_as_float(partner<3>(__float_as_uint(v))));
}

// ---------------------------------------------------------------------------
// A2: certificates of 4 queries per wave (16 lanes per query, lane = depth).
// ---------------------------------------------------------------------------
template <int D, int LOGK, int NW, bool APPROX>
__device__ __forceinline__ void a2_group(Scan2Shared& sh, int j0, int nq, const float (*qrows)[16], QRec* recs, int wcol0,
                                         const int* jlist, int lane
#ifdef GSC_STAMPS
                                         , uint64_t* acc = nullptr, uint64_t* tl = nullptr
#endif
) {
#ifdef GSC_STAMPS
#define ASTAMP(k)                          \
    if (acc) {                             \
        const uint64_t t_ = stamp();       \
        acc[k] += t_ - *tl;                \
        *tl = t_;                          \
    }
#else
#define ASTAMP(k)
#endif
    constexpr int KW = LOGK >= 9 ? LOGK - 9 : 0;  // depths resolved at wave level
    const int l = lane & 15, gbase = lane & ~15;
    const int t = j0 + (lane >> 4);  // query slot (an index into jlist when given)
    const bool qa = t < nq;
    const int tr = qa ? t : j0;  // safe slot for inactive groups
    const int jr = jlist ? jlist[tr] : tr;
    const int jj = jr;
    // global winner over the NW wave records (first wave at the minimum)
    const int wc = wcol0 + jr;
    const uint32_t mw = (l < NW) ? sh.wrec[l][wc].minbits : kInfBits;
    const uint32_t gmin = fmin16(mw);
    const uint32_t nmin = sum16((mw == gmin && l < NW) ? 1u : 0u);
    const int W = (int)min16((mw == gmin && l < NW) ? (uint32_t)l : 99u);
    const int Wv = W < NW ? W : 0;
    const WaveRec& r = sh.wrec[Wv][wc];
    bool tie2;
    const int ls = rec_slot(r, &tie2);
    const int cstar = (Wv * 64 + (r.lanebits & 255)) * 8 + ls;
    const bool tie = nmin > 1 || tie2;
    const float* q = qrows[jr];
    ASTAMP(12)
    // sibling-subtree minimum at depth l
    uint32_t sib = kInfBits;
    if (l < KW) {
        const int sh_ = KW - 1 - l;  // sibling wave group of W at depth l
        const int want = (W >> sh_) ^ 1;
#pragma unroll
        for (int w = 0; w < NW; ++w)
            if ((w >> sh_) == want) sib = fminb(sib, sh.wrec[w][wc].minbits);
    } else if (l < LOGK) {
        const int idx = l <= LOGK - 4 ? (LOGK - 4 - l) : (l == LOGK - 3 ? 8 : (l == LOGK - 2 ? 7 : 6));
        sib = rec_sib(r, ls, idx);
    }
    // split node at depth l on c*'s root path (ANNkd_split::ann_search)
    bool far = false;
    float inc = 0.0f;
    if (l < LOGK) {
        const int h = (1 << l) - 1 + (cstar >> (LOGK - l));
        const bool golo = ((cstar >> (LOGK - 1 - l)) & 1) == 0;
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
    const uint32_t farmask = (uint32_t)(__ballot(far) >> gbase) & 0xFFFFu;
    ASTAMP(13)
    // annBoxDistance(q, enclosing rect): lane l holds dimension l's term (or
    // -1 = inside), summed below in dimension order; box' increments by depth
    {
        float term = -1.0f;
        if (l < D) {
            const float qd = q[l], blo = sh.t.bnd_lo[l], bhi = sh.t.bnd_hi[l];
            const bool below = blo > qd, above = qd > bhi;
            const float t = below ? fsub(blo, qd) : fsub(qd, bhi);
            term = (below || above) ? fmul(t, t) : -1.0f;
        }
        sh.a2s[wave_of_lane()][lane] = term;
        sh.a2i[wave_of_lane()][lane] = inc;
    }
    wave_lds_sync();
    float box = 0.0f;
    {
        const float* tv = &sh.a2s[wave_of_lane()][gbase];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const float v = tv[d];
            box = v >= 0.0f ? fadd(box, v) : box;
        }
    }
    float incs[LOGK];
#pragma unroll
    for (int k = 0; k < LOGK; ++k) incs[k] = sh.a2i[wave_of_lane()][gbase + k];
    wave_lds_sync();  // the scratch is rewritten by this wave's next group
    float bp[LOGK];
#pragma unroll
    for (int k = 0; k < LOGK; ++k) {
        bp[k] = -__builtin_inff();
        if ((farmask >> k) & 1u) {
            box = fadd(box, incs[k]);
            bp[k] = box;
        }
    }
    float Bv = -__builtin_inff(), run = -__builtin_inff();
#pragma unroll
    for (int k = LOGK - 1; k >= 0; --k) {
        run = fmaxf(run, bp[k]);
        Bv = (l == k) ? run : Bv;
    }
    ASTAMP(14)
    const uint32_t m2 = fmin16(sib);  // every leaf except c*
    bool ok, unique;
    float m2lo;
    if constexpr (APPROX) {
        // A1 values are within eps of the reference's distances: certify with margins
        const float qs = l < D ? q[l] : 0.0f;
        const float qn = fsum16(__builtin_fmaf(qs, qs, 0.0f));
        float M = 0.0f;
#pragma unroll
        for (int w = 0; w < NW; ++w) M = fmaxf(M, sh.cnmax[w]);
        const float eps = fadd(fmul(fadd(qn, M), 0x1p-17f), 1e-37f);
        ok = !far || (fsub(fadd(qn, __uint_as_float(sib)), eps) > Bv);
        unique = fsub(__uint_as_float(m2), __uint_as_float(gmin)) > fadd(eps, eps);
        m2lo = fsub(fadd(qn, __uint_as_float(m2)), eps);
    } else {
        ok = !far || (__uint_as_float(sib) > Bv);
        unique = !tie;
        m2lo = __uint_as_float(m2);
    }
    const bool gok = ((__ballot(!ok) >> gbase) & 0xFFFFull) == 0;
    const bool valid = unique && __uint_as_float(gmin) <= FLT_MAX && gok;
    if (qa) {
        QRec& R = recs[jj];
        if (l < LOGK) R.B[l] = Bv;
        if (l == 0) {
            R.valid = valid ? 1 : 0;
            R.cstar = cstar;
            R.id = sh.t.pidx[cstar];
            R.g = __uint_as_float(gmin);  // exact mode only (the solo query); batch queries: vp_end
            R.m2 = m2lo;
            R.rate = sh.rate[cstar];
            R.farmask = farmask;
        }
    }
    ASTAMP(15)
}
#undef ASTAMP

// ---------------------------------------------------------------------------
// Commit, step 1 (wave 0, lanes = queries j of the pending batch): online
// updates in order per centroid (encoder.lpr:735-740, f32 c += (x - c) * rate)
// assuming every query of the batch commits; version table for the checks.
// Log entry e is lane e: position lg_pos (-1 = empty), tag = committing batch.
// ---------------------------------------------------------------------------
// Scan state of one pending query (lane j) / log entry (lane e), built one
// step per A1 query so the LDS round trips hide under wave 0's distance work.
struct VPState {
    int cs, pred, nxt, first, ie;
};

template <int D, int LOGK>
__device__ __forceinline__ void vp_begin(Scan2Shared& sh, int qb, int off, int pn, int a1, int lane, int& lg_pos,
                                         int lg_tag, VPState& st) {
    if (lg_pos >= 0 && lg_tag < a1) lg_pos = -1;  // committed before the batch's snapshot
    st.cs = lane < pn ? sh.qrec[qb][off + lane].cstar : -2;
    st.pred = -1;
    st.nxt = kBatch;
    st.first = kBatch;
    st.ie = 64;
    sh.vpos[lane] = lg_pos;
    sh.vfrom[lane] = 0;
    wave_lds_sync();
}

// step k (uniform): pending query k against every lane's query / entry, all
// in registers (c*_k by readlane, the entries holding it by ballot)
__device__ __forceinline__ void vp_step(int k, int lane, int lg_pos, VPState& st) {
    const int ck = __builtin_amdgcn_readlane(st.cs, k);  // -2 past the batch: matches nothing
    const bool same = ck == st.cs;
    if (k < lane && same) st.pred = 64 + k;
    if (k > lane && same && st.nxt == kBatch) st.nxt = k;
    if (ck == lg_pos && st.first == kBatch) st.first = k;  // lane as log entry: first query moving it
    const uint64_t em = __ballot(lg_pos == ck);            // entries holding c*_k (lowest = ie_k)
    if (lane == k && em) st.ie = __ffsll((long long)em) - 1;
}

// Commit, step 1 (wave 0, lanes = queries j of the pending batch): online
// updates in order per centroid (encoder.lpr:735-740, f32 c += (x - c) * rate)
// assuming every query of the batch commits; version table for the checks.
// Log entry e is lane e: position lg_pos (-1 = empty), tag = commit iteration.
template <int D, int LOGK>
__device__ __forceinline__ void vp_end(Scan2Shared& sh, int qb, int off, int pn, int lane, int lg_pos,
                                       const VPState& st) {
    const int j = lane;
    const bool act = j < pn;
    const QRec& R = sh.qrec[qb][off + (act ? j : 0)];
    const int cs = st.cs, nxt = st.nxt;
    const int ie = st.ie < 64 ? st.ie : -1;  // log entry holding c*_j (c*_j moved before the batch)
    const int pred = st.pred >= 0 ? st.pred : ie;
    // versions: log entries (0..63) and "after query j" (64+j)
    sh.vto[lane] = lg_pos >= 0 ? st.first : -1;
    if (lane < kBatch) {
        sh.vpos[64 + lane] = act ? cs : -1;
        sh.vfrom[64 + lane] = j + 1;
        sh.vto[64 + lane] = act ? nxt : -1;
        sh.nxt[lane] = nxt;
        sh.ient[lane] = ie;
        sh.inval[lane] = 0;
    }
    // chained updates: a query waits for its predecessor's new coordinates
    uint64_t done = ~__ballot(act);
    for (;;) {
        const bool ready = act && !((done >> j) & 1ull) && (pred < 64 || ((done >> (pred - 64)) & 1ull));
        const uint64_t rm = __ballot(ready);
        if (!rm) break;
        if (ready) {
            const float* qv = sh.q[qb][off + j];
            const float* o = pred < 0 ? R.o : (pred < 64 ? sh.lg_c[pred] : sh.newc[pred - 64]);
            float oc[D];
#pragma unroll
            for (int d = 0; d < D; ++d) oc[d] = o[d];
            // exact live distance to c* (its snapshot coordinates when unmoved;
            // the A1 values of the batch are bounds only)
            const float gpj = seqdist<D>(qv, oc);
            const bool okc = R.valid != 0 && (pred < 0 || gpj < R.m2);
            const float rate = R.rate;
#pragma unroll
            for (int d = 0; d < D; ++d) sh.newc[j][d] = fadd(oc[d], fmul(fsub(qv[d], oc[d]), rate));
            sh.gp[j] = gpj;
            if (!okc) sh.inval[j] = 1;
        }
        wave_lds_sync();  // this round's newc feed the next round's lanes
        done |= rm;
    }
}

// Commit, step 2 (all threads): every (query, moved centroid) pair of the
// pending batch -- the moved centroid must stay provably outside ANN's answer.
// Lane = query j (lane & 31); wave / half-wave = a strided share of the
// versions, so each version row is one LDS broadcast per half-wave and the
// query row stays in registers.
template <int D, int LOGK, int NW>
__device__ __forceinline__ void v_check_q(Scan2Shared& sh, int qb, int off, int pn, int wave, int lane) {
    const int j = lane & 31, hf = lane >> 5;
    const bool act = j < pn;
    const int jr = act ? j : 0;
    const QRec& R = sh.qrec[qb][off + jr];
    const int cs = R.cstar;
    const uint32_t fm = R.farmask;
    const float g = sh.gp[jr];
    float q[D];
#pragma unroll
    for (int d = 0; d < D; ++d) q[d] = sh.q[qb][off + jr][d];
    bool bad = false;
#pragma unroll 1
    for (int v = wave * 2 + hf; v < kVer; v += 2 * NW) {
        const int vp = sh.vpos[v];
        if (vp < 0 || !act || j < sh.vfrom[v] || j > sh.vto[v] || vp == cs) continue;
        const float* c = v < 64 ? sh.lg_c[v] : sh.newc[v - 64];
        float du = 0.0f;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const float t = fsub(q[d], c[d]);
            du = fadd(du, fmul(t, t));
        }
        const int lca = __clz(vp ^ cs) - (32 - LOGK);
        const bool farl = (fm >> lca) & 1u;
        if (!(du > g && (!farl || du > R.B[lca]))) bad = true;
    }
    if (bad) sh.inval[j] = 1;
}

template <int D, int LOGK>
__device__ __forceinline__ void v_check(Scan2Shared& sh, int qb, int off, int pn, int tid, int nthreads) {
    const int npairs = pn * kVer;
    for (int p = tid; p < npairs; p += nthreads) {
        const int j = p / kVer, v = p - j * kVer;
        const int vp = sh.vpos[v];
        if (vp < 0 || j < sh.vfrom[v] || j > sh.vto[v]) continue;
        const QRec& R = sh.qrec[qb][off + j];
        const int cs = R.cstar;
        if (vp == cs) continue;  // c* itself: checked in v_prepare
        const float* c = v < 64 ? sh.lg_c[v] : sh.newc[v - 64];
        const float du = seqdist<D>(sh.q[qb][off + j], c);
        const float g = sh.gp[j];
        const int lca = __clz(vp ^ cs) - (32 - LOGK);
        const bool farl = (R.farmask >> lca) & 1u;
        if (!(du > g && (!farl || du > R.B[lca]))) sh.inval[j] = 1;
    }
}

// Exact ANN ann_search (k = 1, eps = 0; annkSearch @0x1800124b0) over the
// stale tree with the live leaf distances in sh.dist -- one lane, stack in
// LDS.  No NaN distances reach this kernel (those passes run the generic
// kernel), so leaf early exits cannot change a result.
// Exact ANN ann_search (k = 1, eps = 0; annkSearch @0x1800124b0) over the
// stale tree with the live leaf distances in sh.dist, for the query in
// sh.qslow.  All threads first tabulate every split node's near child and
// box' increment (ANNkd_split::ann_search: cut = q[cd] - cv; bd = lo - q[cd]
// or q[cd] - hi, clamped at 0; box' = (cut^2 - bd^2) + box), then one lane
// walks the DFS with the stack in LDS.  No NaN distances reach this kernel
// (those passes run the generic kernel), so leaf early exits cannot change a
// result.
template <int D, int LOGK>
__device__ __forceinline__ void dfs_exact(Scan2Shared& sh, int tid, int nthreads) {
    constexpr int K = 1 << LOGK;
    const float* q = sh.qslow;
    for (int h = tid; h < K - 1; h += nthreads) {
        const int cdim = sh.t.cd[h];
        const float qc = q[cdim];
        const float cut = fsub(qc, sh.t.cv[h]);
        const bool nearlo = cut < 0.0f;
        float bd = nearlo ? fsub(sh.t.lo[h], qc) : fsub(qc, sh.t.hi[h]);
        if (bd < 0.0f) bd = 0.0f;
        const float inc = fsub(fmul(cut, cut), fmul(bd, bd));  // >= +0
        sh.dfs_inc[h] = nearlo ? inc : -inc;
    }
    lds_barrier();
    if (tid == 0) {
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
            const float v = sh.dfs_inc[h];
            const int hi = __float_as_uint(v) >> 31;
            sh.st_box[sp] = fadd(cur_box, fabsf(v));
            sh.st_h[sp] = 2 * h + 2 - hi;
            ++sp;
            h = 2 * h + 1 + hi;
        }
        sh.slow_pos = best;
        sh.slow_key = key;
    }
    lds_barrier();
}

// Exact ANN ann_search (k = 1, eps = 0; annkSearch @0x1800124b0), all
// threads: the result of the stale-tree DFS is decided by its strict
// improvements only.  With leaves ranked in near-first DFS order, a leaf is
// reached while the best distance is b iff every far subtree on its path
// entered after the current best was found has box' < b; box' only grows
// along a path, so that is one test on its innermost far subtree (start rank
// s*, box' bx*).  The next improvement is the lowest-ranked reached leaf with
// d < b, found by one block min-reduction per improvement.  Live leaf
// distances come from sh.dist.
template <int D, int LOGK, int NW>
__device__ __forceinline__ void dfs_parallel(Scan2Shared& sh, int tid, int lane, int wave, int& out_pos, float& out_key) {
    constexpr int K = 1 << LOGK;
    constexpr int nthreads = 64 * NW;
    const float* q = sh.qslow;
    for (int h = tid; h < K - 1; h += nthreads) {  // split nodes: box' increment, sign = near child hi
        const int cdim = sh.t.cd[h];
        const float qc = q[cdim];
        const float cut = fsub(qc, sh.t.cv[h]);
        const bool nearlo = cut < 0.0f;
        float bd = nearlo ? fsub(sh.t.lo[h], qc) : fsub(qc, sh.t.hi[h]);
        if (bd < 0.0f) bd = 0.0f;
        const float inc = fsub(fmul(cut, cut), fmul(bd, bd));  // >= +0
        sh.dfs_inc[h] = nearlo ? inc : -inc;
    }
    float rootbox = 0.0f;
#pragma unroll
    for (int d = 0; d < D; ++d) {  // annBoxDistance
        const float qd = q[d];
        if (sh.t.bnd_lo[d] > qd) {
            const float t = fsub(sh.t.bnd_lo[d], qd);
            rootbox = fadd(rootbox, fmul(t, t));
        } else if (qd > sh.t.bnd_hi[d]) {
            const float t = fsub(qd, sh.t.bnd_hi[d]);
            rootbox = fadd(rootbox, fmul(t, t));
        }
    }
    lds_barrier();
    // this lane's 8 leaves (an aligned depth LOGK-3 subtree): DFS rank, start
    // rank and box' of the innermost far subtree (-1 / none if all-near)
    const int p0 = tid * 8;
    int rs[8];  // rank << 13 | (s* + 1)
    float bxs[8];
    {
        float box = rootbox, bF = 0.0f;
        int pref = 0, sF = -1, h = 0;
        for (int l = 0; l < LOGK - 3; ++l) {
            const int bit = (p0 >> (LOGK - 1 - l)) & 1;
            const float v = sh.dfs_inc[h];
            if (bit != (int)(__float_as_uint(v) >> 31)) {
                box = fadd(box, fabsf(v));
                sF = pref + (1 << (LOGK - 1 - l));
                bF = box;
                pref += 1 << (LOGK - 1 - l);
            }
            h = 2 * h + 1 + bit;
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            float box2 = box, bF2 = bF;
            int pref2 = pref, sF2 = sF, h2 = h;
#pragma unroll
            for (int l = LOGK - 3; l < LOGK; ++l) {
                const int bit = ((p0 + s) >> (LOGK - 1 - l)) & 1;
                const float v = sh.dfs_inc[h2];
                if (bit != (int)(__float_as_uint(v) >> 31)) {
                    box2 = fadd(box2, fabsf(v));
                    sF2 = pref2 + (1 << (LOGK - 1 - l));
                    bF2 = box2;
                    pref2 += 1 << (LOGK - 1 - l);
                }
                h2 = 2 * h2 + 1 + bit;
            }
            rs[s] = (pref2 << 13) | (sF2 + 1);
            bxs[s] = bF2;
        }
    }
    // improvements: the empty list takes the first leaf reached (max_key = FLT_MAX)
    int pos = -1, bp = -1, par = 0;
    float b = FLT_MAX;
    for (;;) {
        uint32_t key = 0xFFFFFFFFu;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int rk = rs[s] >> 13, st = (rs[s] & 8191) - 1;
            const bool reach = st <= pos || bxs[s] < b;
            if (p0 + s < K && rk > pos && reach && sh.dist[p0 + s] < b)
                key = min(key, ((uint32_t)rk << 12) | (uint32_t)(p0 + s));
        }
        key = min(key, partner<0>(key));
        key = min(key, partner<1>(key));
        key = min(key, partner<2>(key));
        key = min(key, partner<3>(key));
        key = min(key, partner<4>(key));
        key = min((uint32_t)__builtin_amdgcn_readlane((int)key, 0), (uint32_t)__builtin_amdgcn_readlane((int)key, 32));
        if (lane == 0) sh.wkey[par][wave] = key;
        lds_barrier();
        uint32_t g = 0xFFFFFFFFu;
#pragma unroll
        for (int w = 0; w < NW; ++w) g = min(g, sh.wkey[par][w]);
        par ^= 1;
        if (g == 0xFFFFFFFFu) break;
        pos = (int)(g >> 12);
        bp = (int)(g & 4095u);
        b = sh.dist[bp];
    }
    out_pos = bp;
    out_key = b;
}

// fold published log entries into the owners' registers
template <int D>
__device__ __forceinline__ void refresh(Scan2Shared& sh, float (&creg)[8][D], float (&cn)[8], float& cnmax, int wave,
                                        int lane) {
    const int pp = sh.pub_pos[lane];
    uint64_t m = __ballot(pp >= 0 && (pp >> 9) == wave);
    const bool any = m != 0;
    while (m) {
        const int e = __ffsll((long long)m) - 1;
        m &= m - 1;
        const int p = __builtin_amdgcn_readlane(pp, e);
        const int owner = (p >> 3) & 63, slot = p & 7;
        const float nv = sh.lg_c[e][kRow - 1];  // |c|^2, written with the entry
        // the wave's norm bound only grows within a pass (A2 reads it for any earlier snapshot)
        cnmax = fmaxf(cnmax, nv);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            if (s == slot) {
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const float v = sh.lg_c[e][d];
                    creg[s][d] = lane == owner ? v : creg[s][d];
                }
                cn[s] = lane == owner ? nv : cn[s];
            }
        }
    }
    if (any && lane == 0) sh.cnmax[wave] = cnmax;
}

// c*'s snapshot coordinates for the queries in qmask of batch buffer buf, written by the lane that owns c*
// (the first wave / lane / slot at the minimum of the A1 records, as in A2)
template <int D, int NW>
__device__ __forceinline__ void write_cstar(Scan2Shared& sh, const float (&creg)[8][D], int buf, uint64_t qmask,
                                            int wave, int lane) {
    uint64_t won;
    {
        const bool act = (qmask >> lane) & 1ull;
        const int jq = act ? lane : 0;
        float gm = __builtin_inff();
        int W = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const float m = __uint_as_float(sh.wrec[w][jq].minbits);
            if (m < gm) {
                gm = m;
                W = w;
            }
        }
        won = __ballot(act && W == wave);
    }
    while (won) {
        const int jj = __ffsll((long long)won) - 1;
        won &= won - 1;
        const WaveRec& r = sh.wrec[wave][jj];
        bool tie2;
        const int owner = r.lanebits & 255, slot = rec_slot(r, &tie2);
#pragma unroll
        for (int s = 0; s < 8; ++s)
            if (s == slot && lane == owner) {
#pragma unroll
                for (int d = 0; d < D; ++d) sh.qrec[buf][jj].o[d] = creg[s][d];
            }
    }
}

template <int D, int LOGK>
__global__ __launch_bounds__(512) void scan_batch_kernel(ReduceFrame* __restrict__ frames, int nframes,
                                                         const float* __restrict__ Xall, float* __restrict__ Call,
                                                         int* __restrict__ i_scratch, const float* __restrict__ rate_tab,
                                                         double tol, int max_passes) {
    constexpr int K = 1 << LOGK;
    constexpr int NW = K >= 512 ? K / 512 : 1;
    constexpr int kErrWave = NW > 1 ? 1 : 0;  // residual + cluster ids (wave 0 keeps the log)
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
    int* prev_cnt = uniform_ptr(i_scratch + frp->k_off);  // cnts[not Odd(iter)] by centroid id
    int* cnta = uniform_ptr(i_scratch + frp->ka_off);     // cnts[Odd(iter)] by kd-leaf position
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nthreads = 64 * NW;

    // All of the frame's passes run in this launch (the pass index lives in
    // the frame descriptor), so a frame never waits for the slowest frame of a
    // pass; a NaN pass returns and the generic kernel takes that pass over.
    for (int pass = uniform_int(frp->iters); pass < max_passes; ++pass) {
#ifdef GSC_STAMPS
    const uint64_t t_kernel0 = stamp();
#endif
    if (pass == 0)
        for (int k = tid; k < K; k += nthreads) prev_cnt[k] = 1;  // CCntStart (encoder.lpr:717-721)
    if (tid == 0) sh.any_nan = 0;
    __syncthreads();
    if (!build_tree_fast<D, LOGK, 64 * NW>(sh.t, sh.dist, sh.dfs_inc, C, &sh.slow_pos)) {
        build_tree<D>(sh.t, sh.dist, C, K);  // median ties: quickselect's exact order
        if (tid == 0) frp->tree_exact += 1;
    }

    float creg[8][D];
    float cn[8];  // |c|^2 per register leaf (A1 bounds)
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
            cnta[p] = 1;
        } else {
#pragma unroll
            for (int d = 0; d < D; ++d) creg[s][d] = 0.0f;
        }
        cn[s] = norm2_x<D>(creg[s]);
    }
    if (nan_here) sh.any_nan = 1;
    float cnmax;
    {
        float mx = 0.0f;
#pragma unroll
        for (int s = 0; s < 8; ++s) mx = fmaxf(mx, cn[s]);
        cnmax = wave_max_nonneg(nan_here ? 0.0f : mx);  // NaN passes leave for the generic kernel below
        if (lane == 0) sh.cnmax[wave] = cnmax;
    }
    // first batch's queries
    const int n0 = min(kBatch, N);
    for (int k = tid; k < n0 * D; k += nthreads) {
        const float x = X[k];
        sh.q[0][k / D][k % D] = x;
        sh.qm[0][k / D][k % D] = -2.0f * x;
    }
    __syncthreads();
    if (uniform_int(sh.any_nan)) {
        // NaN centroids (yakmo 0/0 means) make ANN's early exits order dependent:
        // this pass runs in the generic kernel (gsc_kernels.hip)
        if (tid == 0) frp->generic = 1;
        return;
    }

    // wave-0 state: update log (lane = entry, tag = commit iteration) + residual (lane 0)
    int lg_pos = -1, lg_tag = 0;
    double err = 0.0;
    int slow_total = 0, restarts = 0;
#ifdef GSC_STAMPS
    uint64_t acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tlast = stamp();
    acc[9] = tlast - t_kernel0;  // pass setup: tree build, registers, first queries
#endif
    // batches awaiting commit, in order: buffer, first query of the buffer,
    // first uncommitted slot, count, iteration of their distance snapshot
    int vq_buf[2] = {0, 0}, vq_s[2] = {0, 0}, vq_off[2] = {0, 0}, vq_n[2] = {0, 0}, vq_a1[2] = {0, 0};
    int nvq = 0;
    int cur_buf = 0, cur_s = 0, cur_n = n0;  // batch whose distances are computed this iteration
    int next_load = n0;
    for (int it = 0;; ++it) {
        const bool has_p = nvq > 0;
        const int P_buf = vq_buf[0], P_s = vq_s[0], P_off = vq_off[0], P_n = has_p ? vq_n[0] : 0;
        // prefetch the next batch's queries (they land in LDS in part 3)
        constexpr int PE = (kBatch * D + 64 * NW - 1) / (64 * NW);
        float pre[PE];
#pragma unroll
        for (int e = 0; e < PE; ++e) {
            const int k = tid + e * nthreads;
            pre[e] = (k < kBatch * D && next_load + k / D < N) ? X[(int64_t)next_load * D + k] : 0.0f;
        }
        // ---- part 1: chain the pending batch's updates (wave 0); A1(current)
        VPState vst;
        if (wave == 0 && has_p) vp_begin<D, LOGK>(sh, P_buf, P_off, P_n, vq_a1[0], lane, lg_pos, lg_tag, vst);
        STAMP(0)
        // two queries per trip: one query's min-tree (a dependent DPP chain)
        // overlaps the other's distance FMAs
#pragma unroll 1
        for (int jj = 0; jj < cur_n; jj += 2) {
            const int j1 = jj + 1 < cur_n ? jj + 1 : jj;
            float dv0[8], dv1[8];
            a1_dist_x2<D>(creg, cn, sh.qm[cur_buf][jj], sh.qm[cur_buf][j1], dv0, dv1);
            a1_reduce2<LOGK>(dv0, dv1, sh.wrec[wave][jj], sh.wrec[wave][j1], wave, lane);
            if (wave == 0 && has_p) {
                vp_step(jj, lane, lg_pos, vst);
                if (jj + 1 < cur_n) vp_step(jj + 1, lane, lg_pos, vst);
            }
        }
        if (wave == 0 && has_p) {
#pragma unroll 1
            for (int k = cur_n; k < kBatch; ++k) vp_step(k, lane, lg_pos, vst);
            vp_end<D, LOGK>(sh, P_buf, P_off, P_n, lane, lg_pos, vst);
        }
        STAMP(1)
        lds_barrier();
        STAMP(6)
        // ---- part 2: check the pending batch; certificates of the current batch
        if (has_p) v_check_q<D, LOGK, NW>(sh, P_buf, P_off, P_n, wave, lane);
        STAMP(7)
        if (cur_n > 0) {
            // c*'s snapshot coordinates (and exact distance), written by the wave that owns c*
            write_cstar<D, NW>(sh, creg, cur_buf, (1ull << cur_n) - 1ull, wave, lane);
            STAMP(8)
#pragma unroll 1
            for (int j0 = wave * 4; j0 < cur_n; j0 += 4 * NW)
                a2_group<D, LOGK, NW, true>(sh, j0, cur_n, sh.q[cur_buf], sh.qrec[cur_buf], 0, nullptr, lane
#ifdef GSC_STAMPS
                                      , acc, &tlast
#endif
                );
        }
        STAMP(2)
        lds_barrier();
        if (cur_n > 0) {
            // queries the approximate certificate could not decide: exact A1 + A2
            // on the same snapshot (the registers change only in part 4)
            const uint64_t fx = __ballot(lane < cur_n && sh.qrec[cur_buf][lane].valid == 0);
            if (fx) {
                const int nfx = __popcll(fx);
                if (wave == 0 && ((fx >> lane) & 1ull)) sh.fxl[__popcll(fx & ((1ull << lane) - 1ull))] = lane;
                uint64_t m = fx;
                while (m) {
                    const int jj = __ffsll((long long)m) - 1;
                    m &= m - 1;
                    a1_query<D, LOGK>(creg, sh.q[cur_buf][jj], sh.wrec[wave][jj], wave, lane);
                }
                lds_barrier();
                write_cstar<D, NW>(sh, creg, cur_buf, fx, wave, lane);
#pragma unroll 1
                for (int j0 = wave * 4; j0 < nfx; j0 += 4 * NW)
                    a2_group<D, LOGK, NW, false>(sh, j0, nfx, sh.q[cur_buf], sh.qrec[cur_buf], 0, sh.fxl, lane);
                lds_barrier();
            }
        }
        STAMP(3)
        // ---- part 3: commit the valid prefix of the pending batch
        int fj = -1;
        if (has_p) {
            const uint64_t bad = __ballot(lane < P_n && sh.inval[lane] != 0);
            fj = bad ? __ffsll((long long)bad) - 1 : -1;
        }
        if (wave == kErrWave && has_p) {
            // cluster ids, counts and the residual in query order (encoder.lpr:743:
            // err += sqrt(best / colCount)) -- beside wave 0's log update
            const int k = fj >= 0 ? fj : P_n;
            const int j = lane;
            const bool cj = j < k;
            const QRec& R = sh.qrec[P_buf][P_off + (cj ? j : 0)];
            if (cj) {
                clusters[P_s + P_off + j] = R.id;
                atomicAdd(&cnta[R.cstar], 1);
            }
            const float sq = cj ? __fsqrt_rn(sh.gp[j] / (float)D) : 0.0f;
#pragma unroll
            for (int jj = 0; jj < kBatch; ++jj) {
                const double t = (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(sq), jj));
                err = jj < k ? err + t : err;
            }
        }
        if (wave == 0 && has_p) {
            const int k = fj >= 0 ? fj : P_n;
            const int j = lane;
            const bool cj = j < k;
            const QRec& R = sh.qrec[P_buf][P_off + (cj ? j : 0)];
            // the last committed update of each centroid becomes its log entry:
            // the entry already holding that centroid, else the r-th free entry
            const bool lastc = cj && sh.nxt[j] >= k;
            int tgt = lastc ? sh.ient[j] : -1;
            const uint64_t need = __ballot(lastc && tgt < 0);
            const uint64_t freem = __ballot(lg_pos < 0);
            const uint64_t below = (1ull << lane) - 1ull;
            sh.asg[lane] = -1;
            if (lg_pos < 0) sh.freel[__popcll(freem & below)] = lane;
            wave_lds_sync();
            if (lastc && tgt < 0) tgt = sh.freel[__popcll(need & below)];
            if (lastc) {
#pragma unroll
                for (int d = 0; d < D; ++d) sh.lg_c[tgt][d] = sh.newc[j][d];
                sh.lg_c[tgt][kRow - 1] = norm2_x<D>(sh.newc[j]);
                sh.asg[tgt] = R.cstar;
            }
            wave_lds_sync();
            const int a = sh.asg[lane];
            if (a >= 0) {
                lg_pos = a;
                lg_tag = it;
            }
            if (fj >= 0 && lane < D) sh.qslow[lane] = sh.q[P_buf][P_off + fj][lane];
        }
        // queue bookkeeping (uniform)
        const int solo_j = fj >= 0 ? P_s + P_off + fj : -1;
        if (has_p) {
            if (fj >= 0 && fj + 1 < P_n) {
                vq_off[0] = P_off + fj + 1;
                vq_n[0] = P_n - fj - 1;
            } else {
                vq_buf[0] = vq_buf[1];
                vq_s[0] = vq_s[1];
                vq_off[0] = vq_off[1];
                vq_n[0] = vq_n[1];
                vq_a1[0] = vq_a1[1];
                --nvq;
            }
        }
        if (cur_n > 0) {
            vq_buf[nvq] = cur_buf;
            vq_s[nvq] = cur_s;
            vq_off[nvq] = 0;
            vq_n[nvq] = cur_n;
            vq_a1[nvq] = it;
            ++nvq;
        }
        // next batch of distances: into a free buffer, never the buffer a
        // failed query's coordinates are being copied out of (wave 0, above)
        cur_n = 0;
        const int freeb = nvq == 0 ? (fj >= 0 ? P_buf ^ 1 : 0) : (nvq == 1 ? vq_buf[0] ^ 1 : -1);
        if (freeb >= 0 && !(fj >= 0 && freeb == P_buf) && next_load < N) {
            cur_buf = freeb;
            cur_s = next_load;
            cur_n = min(kBatch, N - next_load);
            next_load += cur_n;
#pragma unroll
            for (int e = 0; e < PE; ++e) {
                const int k = tid + e * nthreads;
                if (k < cur_n * D) {
                    sh.q[cur_buf][k / D][k % D] = pre[e];
                    sh.qm[cur_buf][k / D][k % D] = -2.0f * pre[e];
                }
            }
        }
        if (wave == 0) {  // publish this iteration's commits (earlier ones are in the registers)
            const bool fresh_e = lg_pos >= 0 && lg_tag == it;
            sh.pub_pos[lane] = fresh_e ? lg_pos : -1;
        }
        lds_barrier();
        STAMP(4)
        // ---- part 4: fold the log into the registers
        refresh<D>(sh, creg, cn, cnmax, wave, lane);
        if (solo_j >= 0) {
            // the failed query on the live centroids: fresh distances and
            // certificate; exact DFS if the certificate still fails
            ++restarts;
            a1_query<D, LOGK>(creg, sh.qslow, sh.wrec[wave][kBatch], wave, lane);
            lds_barrier();
            if (wave == 0)
                a2_group<D, LOGK, NW, false>(sh, 0, 1, reinterpret_cast<const float(*)[16]>(sh.qslow), &sh.qsolo, kBatch,
                                             nullptr, lane);
            lds_barrier();
            int bpos;
            float key;
            STAMP(10)
            if (uniform_int(sh.qsolo.valid)) {
                bpos = uniform_int(sh.qsolo.cstar);
                key = sh.qsolo.g;
            } else {
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
                // the centroid registers wait in C (pass-start copy, rewritten at pass end)
                // so the DFS has the register file
#pragma unroll
                for (int s = 0; s < 8; ++s)
                    if (p0 + s < K) {
                        const int id = sh.t.pidx[p0 + s];
#pragma unroll
                        for (int d = 0; d < D; ++d) C[(int64_t)id * D + d] = creg[s][d];
                    }
                __asm__ volatile("" ::: "memory");  // the reload below must not be forwarded from the stores
                lds_barrier();  // sh.dist complete
                dfs_parallel<D, LOGK, NW>(sh, tid, lane, wave, bpos, key);
                bpos = uniform_int(bpos);
                __asm__ volatile("" ::: "memory");
#pragma unroll
                for (int s = 0; s < 8; ++s)
                    if (p0 + s < K) {
                        const int id = sh.t.pidx[p0 + s];
#pragma unroll
                        for (int d = 0; d < D; ++d) creg[s][d] = C[(int64_t)id * D + d];
                    }
                ++slow_total;
                STAMP(11)
            }
            // owner publishes c's coordinates; tid 0 moves it (encoder.lpr:735-744);
            // the move enters the log (later batches' snapshots miss it) and the registers
            const int owner = bpos >> 3, slot = bpos & 7;
#pragma unroll
            for (int s = 0; s < 8; ++s)
                if (s == slot && tid == owner) {
#pragma unroll
                    for (int d = 0; d < D; ++d) sh.solo_c[d] = creg[s][d];
                }
            lds_barrier();
            if (wave == kErrWave && lane == 0) err += (double)__fsqrt_rn(key / (float)D);
            if (wave == 0) {
                if (lane == 0) {
                    const float rate = sh.rate[bpos];
                    for (int d = 0; d < D; ++d) {
                        const float o = sh.solo_c[d];
                        sh.solo_c[d] = fadd(o, fmul(fsub(sh.qslow[d], o), rate));
                    }
                    atomicAdd(&cnta[bpos], 1);
                    clusters[solo_j] = sh.t.pidx[bpos];
                }
                wave_lds_sync();
                const uint64_t hit = __ballot(lg_pos == bpos);
                const int e = hit ? __ffsll((long long)hit) - 1 : __ffsll((long long)__ballot(lg_pos < 0)) - 1;
                if (lane == e) {
                    lg_pos = bpos;
                    lg_tag = it;
#pragma unroll
                    for (int d = 0; d < D; ++d) sh.lg_c[e][d] = sh.solo_c[d];
                    sh.lg_c[e][kRow - 1] = norm2_x<D>(sh.solo_c);
                }
                sh.pub_pos[lane] = lane == e ? bpos : -1;
            }
            lds_barrier();
            refresh<D>(sh, creg, cn, cnmax, wave, lane);
        }
        STAMP(5)
        if (nvq == 0 && cur_n == 0) {
            if (tid == 0) frp->loop_iters = it + 1;
            break;
        }
        if (it > 4 * N + 64) {  // progress guard: every iteration commits or computes
            if (tid == 0) frp->loop_iters = -1;
            break;
        }
    }
    if (wave == kErrWave && lane == 0) sh.err_out = err;
    __syncthreads();
    err = sh.err_out;
    // write back the live centroids and this pass's counts (cnts[Odd(iter)])
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const int p = p0 + s;
        if (p < K) {
            const int id = sh.t.pidx[p];
#pragma unroll
            for (int d = 0; d < D; ++d) C[(int64_t)id * D + d] = creg[s][d];
            // the commits' atomics live in L2: read past this CU's L1
            prev_cnt[id] = __hip_atomic_load(&cnta[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
#ifdef GSC_STAMPS
    if (lane == 0)
        for (int k = 0; k < 16; ++k) frp->stamps[wave * 16 + k] += acc[k];
#endif
    if (tid == 0) {
        const double prev_err = pass == 0 ? 3.4028234663852886e+38 : frp->err;  // err := MaxSingle
        const double diff = err > prev_err ? err - prev_err : prev_err - err;
        frp->iters = pass + 1;
        frp->slow += slow_total;
        frp->restarts += restarts;
        frp->err = err;
        frp->done = (diff <= tol || pass + 1 >= kMaxScanIters || frp->loop_iters < 0) ? 1 : 0;
        sh.pass_done = frp->done;
    }
    // the next pass's tree build and rate lookups read C and prev_cnt as
    // written above by other lanes: agent fence (L1 invalidate) + barrier
    __threadfence();
    __syncthreads();
    if (uniform_int(sh.pass_done)) break;
    }
}

}  // namespace gsc

using namespace gsc;

// Batched KNNScanReduce for every frame (K = 2^logk, 256..4096, D = 8 or 16):
// each frame runs its passes from frp->iters until it converges, reaches
// max_passes or meets a NaN pass (left to the generic kernel).  Returns
// hipErrorInvalidValue for shapes it does not cover.
extern "C" hipError_t gsc_launch_scan_batch(int D, int logk, ReduceFrame* frames, int nframes, const float* X,
                                            float* C, int* is, const float* rate_tab, double tol, int max_passes,
                                            hipStream_t st) {
    const int K = 1 << logk;
    const int threads = 64 * (K >= 512 ? K / 512 : 1);
    const size_t shm = sizeof(Scan2Shared);
#define SB(DV, LK)                                                                                                     \
    if (D == DV && logk == LK) {                                                                                       \
        (void)hipFuncSetAttribute((const void*)scan_batch_kernel<DV, LK>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  (int)shm);                                                                           \
        hipLaunchKernelGGL((scan_batch_kernel<DV, LK>), dim3(nframes), dim3(threads), shm, st, frames, nframes, X, C,   \
                           is, rate_tab, tol, max_passes);                                                                   \
        return hipGetLastError();                                                                                      \
    }
    SB(8, 8) SB(8, 9) SB(8, 10) SB(8, 11) SB(8, 12)
    SB(16, 8) SB(16, 9) SB(16, 10) SB(16, 11) SB(16, 12)
#undef SB
    return hipErrorInvalidValue;
}

extern "C" size_t gsc_scan_batch_shared_bytes(void) { return sizeof(Scan2Shared); }
