// KNNScanReduce (encoder.lpr:699-765) as a batched, speculative pipeline --
// the hot kernel of the SoundChunks encode path.
//
// Reference semantics: per pass, ANN builds a kd-tree over the centroids
// (ann_kdtree_create, encoder.lpr:729) and then, for every point i in order,
// runs an exact k = 1 search on that *stale* tree with the *live* centroids
// (the tree keeps the caller's row pointers; encoder.lpr:733) and moves the
// found centroid towards the point (encoder.lpr:735-744).  Point i+1 sees the
// update of point i, so the chain is sequential.  Only ONE centroid moves per
// point, which is what this kernel exploits.
//
// Layout: the K = 2^LOGK centroids live in VGPRs, SL consecutive kd-leaf
// positions per lane, so every kd subtree is an aligned block of (virtual)
// waves, lanes and slots: leaf position p = (vwave*64 + lane)*SL + slot.
//   D <= 16 (ChunkSize <= 8): one CU per frame, SL = 8 (K = 4096: 8 waves x
//            64 lanes x 8 leaves x D floats).
//   D = 32 (ChunkSize 9 .. 16): 4096 x 32 floats are 512 KB, the whole register
//            file of a CU, so K = 4096 runs the split layout on one CU: the DCT
//            half (DR = 16 features) in VGPRs, the cepstrum half in a per-frame
//            tail array in HBM that only the lane owning a leaf reads and writes.
//            K <= 2048 at D = 32 keeps every feature in VGPRs.
// (Two CUs per frame -- each holding half the leaves, A1 records and
// coordinates exchanged through L2 -- was measured against one CU per frame on
// launches with fewer frames than CUs and removed: 1.4-1.9x slower)
//
// Pipeline, per iteration (batches of KB queries; "current" = the batch
// whose distances are computed now, "pending" = the previous batch, whose
// speculative answers are committed now):
//   part 1  A1 (all waves): snapshot distance bounds of the current batch;
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
// if it fails on a fresh snapshot it is resolved by the exact parallel DFS
// (dfs_parallel) over live distances.
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

#ifndef GSC_DFS_CALL_D
#define GSC_DFS_CALL_D 8  // feature widths whose exact DFS is an out-of-line call (A/B switch)
#endif
#ifndef GSC_VP_EARLY_D
#define GSC_VP_EARLY_D 32  // widest D whose update chain runs right after its prep (A/B switch, see kVpEarly)
#endif
#ifndef GSC_INBATCH_DFS_D
#define GSC_INBATCH_DFS_D 16  // widest D whose uncertified batch queries run the in-batch DFS (D = 32: +0.8 % C3 scan, its split-layout exact distances read the tail rows)
#endif
#ifndef GSC_EPSF8
#define GSC_EPSF8 0x1p-18f  // A1 bound slack at D = 8 (< 56u of its 64u, see a1_dist_x2)
#endif

// Shape of one KNNScanReduce pipeline instance.
template <int D_, int LOGK_, int SL_, int DR_ = D_>
struct ScanCfg {
    static constexpr int D = D_, LOGK = LOGK_, SL = SL_;
    // features held in VGPRs; the other TL (split layout: the cepstrum half)
    // live in a per-frame, position-indexed HBM array that only the lane owning
    // the position reads and writes
    static constexpr int DR = DR_, TL = D_ - DR_;
    static constexpr bool SPLIT = TL > 0;
    static constexpr int K = 1 << LOGK;
    static constexpr int LS = SL == 8 ? 3 : (SL == 4 ? 2 : (SL == 2 ? 1 : 0));  // log2 slots per lane
    static constexpr int LPW = 64 * SL;                                 // leaves per wave
    static constexpr bool FULL = K >= LPW;                              // every lane holds SL leaves
    static constexpr int NWL = FULL ? K / LPW : 1;                      // waves per workgroup
    static constexpr int NWV = NWL;                                     // waves holding leaves
    static constexpr int NT = 64 * NWL;                                 // threads per workgroup
    static constexpr int KW = LOGK - 6 - LS >= 0 ? LOGK - 6 - LS : 0;   // kd depths resolved at wave level
    static constexpr int KB = D > 16 ? 16 : 32;                         // queries per speculative batch
    static constexpr int KVER = 64 + KB;                                // centroid versions a pending batch sees
    // query row stride: odd x 16 B at D >= 16, so per-lane rows (box bounds, V check,
    // update chain) read without b128 bank conflicts (C2 scan -1.0 %: 3332 vs 3366 ms)
    static constexpr int QD = D < 16 ? 16 : D + 4;
    static constexpr int H = D / 2;  // DCT half of the features; [H, D) = cepstrum x 1e-5 (encoder.lpr:1700-1716)
    static constexpr int ROW = D + 4;  // lane-indexed coordinate rows: 16-B multiple, odd x 16 B (no b128 conflicts)
    // A1 bound slack: eps(q) = (|q|^2 + M) * 2^-EPSX (see a1_dist_x2)
    static constexpr float EPSF = D > 16 ? 0x1p-16f : (D > 8 ? 0x1p-17f : GSC_EPSF8);
    static_assert(NWV <= 16, "A2 evaluates up to 16 wave records per query (one per lane of a 16-lane group)");
    static_assert(KB <= 32 && 64 % KB == 0, "batch size");
    static_assert(!SPLIT || DR == H, "split layout: the DCT half in registers");
};

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

template <int SL>
struct WaveRecT {     // A1 output per (wave, query): raw values of the argmin lane L;
                      // the winner's path minima are derived in A2 (rec_* below)
    uint32_t minbits; // wave minimum distance (f32 bits)
    int lanebits;     // L | 256 if another lane of the wave also holds the minimum
    uint32_t sl[6];   // lane L's sibling lane-group minima, groups of 2^b lanes (b = 0..5), as order keys
    uint32_t b[SL];   // lane L's SL leaf values (slots = kd leaves SL*L .. SL*L + SL-1 of the wave)
    // (padding the record to an odd word count for conflict-free column reads
    // was measured and not kept: 3827 vs 3713 ms, the single-lane record
    // stores lose their 16-byte alignment)
};

// first slot of lane L at the wave minimum, and whether another slot ties it
template <int SL>
__device__ __forceinline__ int rec_slot(const WaveRecT<SL>& r, bool* tie2) {
    int ls = SL - 1, lc = 0;
#pragma unroll
    for (int s = SL - 1; s >= 0; --s) {
        const bool e = r.b[s] == r.minbits;
        lc += e ? 1 : 0;
        ls = e ? s : ls;
    }
    *tie2 = lc > 1 || (r.lanebits >> 8) != 0;
    return ls;
}

// sibling-subtree minimum on the path to slot ls: lane groups (idx 0..5),
// sibling slot (6), other slot pair (7), other quad (8, SL = 8 only)
template <int SL>
__device__ __forceinline__ uint32_t rec_sib(const WaveRecT<SL>& r, int ls, int idx) {
    if (idx < 6) return keybits((int)r.sl[idx]);
    if constexpr (SL >= 2) {
        if (idx == 6) return r.b[ls ^ 1];
    }
    if constexpr (SL >= 4) {
        if (SL == 4 || idx == 7) {
            const int pb = (ls & (SL - 4)) | ((ls & 2) ^ 2);
            return fminb(r.b[pb], r.b[pb + 1]);
        }
        const int qb = (ls & 4) ^ 4;
        return fminb(fminb(r.b[qb], r.b[qb + 1]), fminb(r.b[qb + 2], r.b[qb + 3]));
    }
    return kInfBits;  // no slot levels below SL
}

// improvements of ANN's DFS kept per query for the in-batch DFS answers (valid
// == 2 below): a DFS with more keeps its query uncertified (solo resolution)
#ifndef GSC_MAX_IMP
#define GSC_MAX_IMP 8
#endif
constexpr int kMaxImp = GSC_MAX_IMP;

template <int D>
struct QRecT {        // A2 output per query
    int valid;        // 1: certified (A2), 2: ANN's answer on the snapshot by the exact DFS, 0: neither
    int cstar;        // kd-leaf position of the certified answer
    int id;           // centroid id (pidx[cstar])
    float g;          // snapshot distance to c*
    float m2;         // snapshot minimum over every other leaf
    float rate;       // Single(1/sqrt(previous-pass count of c*))
    uint32_t farmask; // far steps on c*'s root path, bit = depth
    int pad_;         // 1: NaN-first query (ANN answers the NaN leaf its descent reaches)
    float B[16];      // suffix max of box' over far steps (certificate thresholds);
                      // valid == 2 (DFS answer): B[i] = the i-th improvement's distance
    float o[D];       // c*'s snapshot coordinates
    int nimp;         // valid == 2: improvements of the snapshot DFS (the last one is c*)
    int ir[kMaxImp];  // valid == 2: improvement i as DFS rank << 12 | kd-leaf position
};

template <class C>
struct Scan2Shared {
    KdTree t;
    // tree build scratch and the exact DFS's live distances share the bytes of
    // the A1 records: the records are dead at pass start and once the solo
    // query's certificate has failed
    union {
        float dist[kMaxK];
        WaveRecT<C::SL> wrec[C::NWV][C::KB + 1];  // column KB: the solo query
    };
    float rate[kMaxK];     // Single(1/sqrt(cnts[not Odd(iter)])) by kd-leaf position
    float dfs_inc[kMaxK];  // exact DFS: per split node box' increment, sign = near child hi
    uint32_t dfs_near[kMaxK / 32];  // NaN passes' exact DFS: near child of split node h is low (bit h)
    alignas(16) float q[2][C::KB][C::QD];
    alignas(16) float qm[2][C::KB][C::QD];  // -2 q (exact), the A1 dot-product operand
    float cnmax[C::NWV];   // per (virtual) wave: upper bound of |c|^2 over its live centroids (monotone within a pass)
    // half-dimension A1 (see a1_dist_x2): per-wave |c_h|^2 / |c|^2 maxima and
    // tail-dimension boxes at pass start, the frame's data tail box (order keys)
    float cnmax_h[C::NWV], cnmax_f[C::NWV];
    float ptlo[C::NWV][C::D], pthi[C::NWV][C::D];
    int xtlo[C::D], xthi[C::D];
    // A1 pruning (one-CU frames): per wave the bounding box of its centroids'
    // live register coordinates (grown by every fold), per batch query an
    // upper bound of the snapshot's minimum distance
    float wlo[C::NWV][C::D], whi[C::NWV][C::D];
    uint32_t ub[C::KB];
    int fxl[C::KB];        // queries of the current batch re-certified exactly
    alignas(16) float qslow[C::QD];  // the query resolved on its own after a failed commit
    alignas(16) QRecT<C::D> qrec[2][C::KB];
    QRecT<C::D> qsolo;
    // update log: entry e = wave-0 lane e (position in a VGPR, coordinates here)
    alignas(16) float lg_c[64][C::ROW];
    int pub_pos[64];       // log entries to fold into the registers (position, -1 = none)
    alignas(16) float solo_c[C::ROW];  // coordinates of the solo query's centroid
    double err_out;
    // commit of the pending batch: versions 0..63 = log entries, 64+j = after query j
    int vcs[C::KB];        // c* of the pending batch's queries (-2 past the batch)
    // per version: x = leaf position (-1 = none), y = first query that sees it,
    // z = last query that sees it (one 16-B read per version in the V check)
    alignas(16) int4 vmeta[C::KVER];
    // new coordinates after each pending query's update and the next query with
    // the same c*, by iteration parity: the waves fold from them after the
    // commit decision while wave 0 may already run the next iteration's chain
    alignas(16) float newc[2][C::KB][C::ROW];
    float gp[C::KB];       // live d(q_j, c*_j)
    int inval[C::KB];
    int nxt[2][C::KB];     // next query of the batch with the same c* (KB = none), by iteration parity
    int ient[C::KB];       // log entry holding c*_j when the commit starts (-1 = none)
    int vie[C::KB];        // vp_begin: log entry holding c*_j (64 = none)
    int freel[64];         // commit: free log entries, in lane order
    int asg[64];           // commit: log entry -> centroid position it now holds
    int slow_pos;
    float slow_key;
    int vc_next;           // V check: next trip to take (reset in part 3)
    int vp_ready;          // V check: iteration + 1 whose update chain (vp_end) is complete
    int any_nan;
    int nan_rows;          // the pass has NaN centroids (yakmo 0/0 means): see nan_first below
    uint32_t nanid[kMaxK / 32];  // centroid id -> NaN row (fixed for the whole pass)
    int pass_done;         // end of pass: the frame converged (or hands the next pass over)
    uint32_t wkey[2][C::NWL];  // parallel exact DFS: per-wave next-improvement keys
    alignas(16) float a2s[C::NWL][C::D > 16 ? 2 : 1][64];  // A2 scratch per wave: box terms by dimension
    alignas(16) float a2i[C::NWL][64];                     // box' increments by depth
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

// the lane index as a value the compiler cannot see through: refreshed at the
// phase boundaries of the scan loop, so every per-lane LDS address is computed
// where it is used (one VALU op) instead of being hoisted out of the loop,
// kept live through A1 and spilled to scratch (a scratch reload is a
// vector-memory round trip, and its vmcnt wait also waits for the query
// prefetch from HBM)
__device__ __forceinline__ int opaque_v(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

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
// A1 pruning.  ANN's DFS reaches ~170 of the 4096 leaves per search on the
// benchmark data; the batched A1 evaluates all of them.  A wave can skip a
// query when no leaf of its 512 can be the answer: lb = box distance from q
// to the bounding box of the wave's centroids (their live register values,
// the box grown at every fold) is a lower bound of every leaf distance there,
// so lb > ub + 4 eps, with ub >= the snapshot's minimum distance, proves the
// wave holds neither c* nor a leaf within the certificate's margins.  ub comes
// from the query's home waves (those whose box contains q: lb = 0), which
// evaluate first; the others decide after one barrier.  (Homes by kd descent
// instead of boxes cover the ~20 % of queries outside every box, but cost the
// kernel 30 more spilled VGPRs and were slower: 5464 vs 5285 ms.)  A skipped wave's
// record carries a valid lower bound of its A1 values instead of a minimum:
//   approximate records (s~ = d~ - |q|^2):  v = (lb - 3 eps) - |q|^2,
//   exact records (fixups):                 v = lb,
// so every certificate inequality A2 evaluates with it stays sound (the
// bound only stands in for minima of other waves and never wins).
// Rounding: lb is a sequential f32 sum (relative error < (D+2) u), scaled by
// (1 - 2^-17) below the real box distance, which is <= every exact f32
// distance scaled by 1 + (D+1) u; eps >= 2^-5 x the roundings of the bound
// arithmetic (|lb|, |q|^2, |d~| <= 2 (|q|^2 + M)).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int wave_min_i(int v) {
    v = min(v, (int)partner<0>((uint32_t)v));
    v = min(v, (int)partner<1>((uint32_t)v));
    v = min(v, (int)partner<2>((uint32_t)v));
    v = min(v, (int)partner<3>((uint32_t)v));
    v = min(v, (int)partner<4>((uint32_t)v));
    return min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 32));
}
__device__ __forceinline__ int wave_max_i(int v) {
    v = max(v, (int)partner<0>((uint32_t)v));
    v = max(v, (int)partner<1>((uint32_t)v));
    v = max(v, (int)partner<2>((uint32_t)v));
    v = max(v, (int)partner<3>((uint32_t)v));
    v = max(v, (int)partner<4>((uint32_t)v));
    return max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 32));
}

// pass start: the box of this wave's leaves
template <class C>
__device__ __forceinline__ void wave_box_init(Scan2Shared<C>& sh, const float (&creg)[C::SL][C::DR], int vwave, int lane,
                                              int p0, uint32_t dmask) {
    if constexpr (C::SPLIT) {  // the tail features: the pass setup's per-wave tail box
        if (lane == 0)
            for (int d = C::DR; d < C::D; ++d) {
                sh.wlo[vwave][d] = sh.ptlo[vwave][d];
                sh.whi[vwave][d] = sh.pthi[vwave][d];
            }
    }
#pragma unroll  // static register indices: a runtime d would demote creg to scratch
    for (int d = 0; d < C::DR; ++d) {
        float lo = __builtin_inff(), hi = -__builtin_inff();
#pragma unroll
        for (int s = 0; s < C::SL; ++s)
            if (!((dmask >> s) & 1u)) {
                lo = fminf(lo, creg[s][d]);
                hi = fmaxf(hi, creg[s][d]);
            }
        const int klo = wave_min_i(ordkey(__float_as_uint(lo)));
        const int khi = wave_max_i(ordkey(__float_as_uint(hi)));
        if (lane == 0) {
            sh.wlo[vwave][d] = __uint_as_float(keybits(klo));
            sh.whi[vwave][d] = __uint_as_float(keybits(khi));
        }
    }
}

// lower bound of every exact leaf distance in wave w's box (0 inside the box)
template <class C>
__device__ __forceinline__ float wave_box_lb(const Scan2Shared<C>& sh, const float* __restrict__ q, int w) {
    float lb = 0.0f;
#pragma unroll
    for (int d = 0; d < C::D; ++d) {
        // branch-free: lo - qd > 0 below the box, qd - hi > 0 above it, else 0
        // (an empty box, lo = +inf > hi = -inf, gives +inf either way); the
        // selected difference is the same f32 value as a branchy select
        const float qd = q[d], lo = sh.wlo[w][d], hi = sh.whi[w][d];
        const float t = fmaxf(fmaxf(fsub(lo, qd), fsub(qd, hi)), 0.0f);
        lb = fadd(lb, fmul(t, t));
    }
    return fmul(lb, 1.0f - 0x1p-17f);
}

// ---------------------------------------------------------------------------
// A1: snapshot distances of one query against this wave's leaves.
// ---------------------------------------------------------------------------
template <int D, int SL>
__device__ __forceinline__ void a1_dist(const float (&creg)[SL][D], const float* __restrict__ qv, float (&dv)[SL]) {
    // ANN leaf distance (ANN.dll @0x1800128b0): dist = dist + (q[d]-p[d])^2, d = 0..D-1
#pragma unroll
    for (int s = 0; s < SL; ++s) dv[s] = 0.0f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float qd = qv[d];
#pragma unroll
        for (int s = 0; s < SL; ++s) {
            const float t = fsub(qd, creg[s][d]);
            dv[s] = fadd(dv[s], fmul(t, t));
        }
    }
}

// wave min-tree over the lanes' SL leaf distances -> the query's WaveRec
template <int SL>
struct A1Tree {
    uint32_t b[SL];  // this lane's leaf values (f32 bits)
    uint32_t lmin;
    int sl[6];       // partner lane-group minima (order keys)
    uint64_t m;      // lanes at the wave minimum
};

template <class C>
__device__ __forceinline__ A1Tree<C::SL> a1_tree(const float (&dv)[C::SL], int vwave, int lane) {
    constexpr int SL = C::SL;
    const int p0 = (vwave * 64 + lane) * SL;
    A1Tree<SL> t;
    const bool has = C::FULL || p0 < C::K;  // small K: only the low lanes hold leaves
#pragma unroll
    for (int s = 0; s < SL; ++s) t.b[s] = has ? __float_as_uint(dv[s]) : kInfBits;
    if constexpr (SL == 1) {
        t.lmin = t.b[0];
    } else {
        uint32_t mm[SL / 2];
#pragma unroll
        for (int s = 0; s < SL / 2; ++s) mm[s] = fminb(t.b[2 * s], t.b[2 * s + 1]);
        if constexpr (SL == 8) {
            t.lmin = fminb(fminb(mm[0], mm[1]), fminb(mm[2], mm[3]));
        } else if constexpr (SL == 4) {
            t.lmin = fminb(mm[0], mm[1]);
        } else {
            t.lmin = mm[0];
        }
    }
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

template <int SL>
__device__ __forceinline__ void a1_store(const A1Tree<SL>& t, WaveRecT<SL>& rec, int lane) {
    const int L = __ffsll((long long)t.m) - 1;
    if (lane == L) {
        rec.minbits = t.lmin;
        rec.lanebits = L | (__popcll(t.m) > 1 ? 256 : 0);
#pragma unroll
        for (int i = 0; i < 6; ++i) rec.sl[i] = (uint32_t)t.sl[i];
#pragma unroll
        for (int s = 0; s < SL; ++s) rec.b[s] = t.b[s];
    }
}

template <class C>
__device__ __forceinline__ void a1_reduce(const float (&dv)[C::SL], WaveRecT<C::SL>& rec, int vwave, int lane) {
    a1_store<C::SL>(a1_tree<C>(dv, vwave, lane), rec, lane);
}

// two queries: both DPP chains are computed before either record store, so
// their latencies overlap
template <class C>
__device__ __forceinline__ void a1_reduce2(const float (&dv0)[C::SL], const float (&dv1)[C::SL], WaveRecT<C::SL>& rec0,
                                           WaveRecT<C::SL>& rec1, int vwave, int lane) {
    const A1Tree<C::SL> t0 = a1_tree<C>(dv0, vwave, lane);
    const A1Tree<C::SL> t1 = a1_tree<C>(dv1, vwave, lane);
    a1_store<C::SL>(t0, rec0, lane);
    a1_store<C::SL>(t1, rec1, lane);
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

// min over the wave of a non-negative float (+inf allowed)
__device__ __forceinline__ float wave_min_nonneg(float x) {
    uint32_t k = __float_as_uint(x);
    k = min(k, partner<0>(k));
    k = min(k, partner<1>(k));
    k = min(k, partner<2>(k));
    k = min(k, partner<3>(k));
    k = min(k, partner<4>(k));
    k = min((uint32_t)__builtin_amdgcn_readlane((int)k, 0), (uint32_t)__builtin_amdgcn_readlane((int)k, 32));
    return __uint_as_float(k);
}

template <class C>
__device__ __forceinline__ void a1_query(const float (&creg)[C::SL][C::DR], const float* __restrict__ qv,
                                         WaveRecT<C::SL>& rec, int vwave, int lane, uint32_t dmask,
                                         const float* __restrict__ trow = nullptr, int p0 = 0, float tw = 0.0f) {
    float dv[C::SL];
    a1_dist<C::DR, C::SL>(creg, qv, dv);
    if constexpr (C::SPLIT) {
        // the reference's sum continued over the tail features, for the leaves
        // that can hold the wave minimum: every partial sum over the first DR
        // features is <= the full one, and the full sum of the leaf at the
        // partial minimum mh is <= U = (mh + TW)(1 + 2^-18); a leaf above U
        // keeps its partial sum -- a lower bound, above the minimum, never tied
        float ml = __builtin_inff();
#pragma unroll
        for (int s = 0; s < C::SL; ++s) ml = ((dmask >> s) & 1u) ? ml : fminf(ml, dv[s]);
        const float U = fmul(fadd(wave_min_nonneg(ml), tw), 1.0f + 0x1p-18f);
#pragma unroll
        for (int s = 0; s < C::SL; ++s)
            if (!((dmask >> s) & 1u) && dv[s] <= U) {
                const float* tr = trow + (int64_t)(p0 + s) * C::TL;
                float a = dv[s];
#pragma unroll
                for (int d = 0; d < C::TL; ++d) {
                    const float t = fsub(qv[C::DR + d], tr[d]);
                    a = fadd(a, fmul(t, t));
                }
                dv[s] = a;
            }
    }
#pragma unroll
    for (int s = 0; s < C::SL; ++s) dv[s] = ((dmask >> s) & 1u) ? __builtin_inff() : dv[s];  // padding leaves
    a1_reduce<C>(dv, rec, vwave, lane);
}

// ---------------------------------------------------------------------------
// A1 of the batch queries: expanded-form distance bounds instead of the exact
// sums.  A1 keeps s~ = |c|^2 + sum_d fma(-2 q_d, c_d, .) per leaf (D VALU ops
// instead of 3D; the wave min-tree runs in float order); A2 adds |q|^2 once.
// d~ = fl(|q|^2 + s~) differs from the reference's sequential f32 distance d
// (ANN.dll @0x1800128b0) by at most eps(q) = (|q|^2 + M) * EPSF, with
// M >= |c|^2 over the live centroids: the D fma roundings are <= 2D u(|c|^2 +
// |q|^2) (every partial sum is within 2(|c|^2 + |q|^2) by Cauchy-Schwarz), the
// two norms <= D u each, the final add <= 2u, the reference's own sum <=
// (D+1) u d <= 2(D+1) u (|c|^2 + |q|^2); u = 2^-24.  D = 16: < 104u against
// the 128u of 2^-17; D = 32: < 200u against the 256u of 2^-16; D = 8: < 56u
// against the 64u of 2^-18 (D = 8 used 2^-17 before round 4: the halved slack
// sends fewer certificates to the exact fixup, C5 -cs4 scan -3 %).  A2 certifies
// only with that margin; what it cannot decide is re-run exactly on the same
// snapshot (fixup in part 2).  The committed distance g is always recomputed
// exactly from c*'s coordinates (vp_end).
// ---------------------------------------------------------------------------
//
// Half-dimension bounds (per pass, one-CU frames): the features [H, D) are the
// cepstrum scaled by 1e-5 (encoder.lpr:1700-1716), so their share of any
// distance is at most TW = sum_{d >= H} (hi_d - lo_d)^2 over the box of the
// frame's data and the pass's centroids (every centroid stays in that box: a
// move is c + (x - c) * rate with rate <= 1, widened by an ulp slack).  With
// DD = H the bound covers the first H features only; the certificate then uses
// |q_h|^2 + TW/2 for |q|^2 and eps + TE for eps, TE = TW/2 + EPSF * (tail
// norms), which keeps every inequality of A2 and of the pruning sound.  A pass
// uses it only when TE is small against the norm scale of eps (else the full
// D-dimension bound, as before).
// ---------------------------------------------------------------------------
template <int DD, int D, int SL>
__device__ __forceinline__ void a1_dist_x2(const float (&creg)[SL][D], const float (&cn)[SL],
                                           const float* __restrict__ qm0, const float* __restrict__ qm1,
                                           float (&dv0)[SL], float (&dv1)[SL]) {
#pragma unroll
    for (int s = 0; s < SL; ++s) {
        dv0[s] = cn[s];
        dv1[s] = cn[s];
    }
#pragma unroll
    for (int d = 0; d < DD; ++d) {
        const float m0 = qm0[d], m1 = qm1[d];
#pragma unroll
        for (int s = 0; s < SL; ++s) {
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

__device__ __forceinline__ float fsum16(float v) {  // sum over each aligned 16-lane row, uniform result
    v = fadd(v, __uint_as_float(partner<0>(__float_as_uint(v))));
    v = fadd(v, __uint_as_float(partner<1>(__float_as_uint(v))));
    v = fadd(v, __uint_as_float(partner<2>(__float_as_uint(v))));
    return fadd(v, __uint_as_float(partner<3>(__float_as_uint(v))));
}

// ---------------------------------------------------------------------------
// A2: certificates of 4 queries per wave (16 lanes per query, lane = depth).
// ---------------------------------------------------------------------------
template <class C, bool APPROX>
__device__ __forceinline__ void a2_group(Scan2Shared<C>& sh, int j0, int nq, const float (*qrows)[C::QD],
                                         QRecT<C::D>* recs, int wcol0, const int* jlist, int lane,
                                         bool half = false, float twh = 0.0f, float te = 0.0f, bool nanpass = false
#ifdef GSC_STAMPS
                                         , uint64_t* acc = nullptr, uint64_t* tl = nullptr, uint64_t* xc = nullptr
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
    constexpr int D = C::D, LOGK = C::LOGK, NW = C::NWV, SL = C::SL, LS = C::LS;
    constexpr int KW = C::KW;  // depths resolved at wave level
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
    const WaveRecT<SL>& r = sh.wrec[Wv][wc];
    bool tie2;
    const int ls = rec_slot<SL>(r, &tie2);
    const int cstar = (Wv * 64 + (r.lanebits & 255)) * SL + ls;
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
        // lane levels: depths [KW, LOGK - LS) -> sibling lane groups 5..0;
        // slot levels: depths [LOGK - LS, LOGK) -> 8 (quad), 7 (pair), 6 (slot)
        const int idx = l < LOGK - LS ? (LOGK - LS - 1 - l) : (6 + (LOGK - 1 - l));
        sib = rec_sib<SL>(r, ls, idx);
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
    // annBoxDistance(q, enclosing rect): lane l holds dimension l's term (and
    // l + 16's at D = 32; -1 = inside), summed below in dimension order; box'
    // increments by depth
    constexpr int NH = D > 16 ? 2 : 1;
    {
#pragma unroll
        for (int hh = 0; hh < NH; ++hh) {
            const int dd = l + 16 * hh;
            float term = -1.0f;
            if (dd < D) {
                const float qd = q[dd], blo = sh.t.bnd_lo[dd], bhi = sh.t.bnd_hi[dd];
                const bool below = blo > qd, above = qd > bhi;
                const float tt = below ? fsub(blo, qd) : fsub(qd, bhi);
                term = (below || above) ? fmul(tt, tt) : -1.0f;
            }
            sh.a2s[wave_of_lane()][hh][lane] = term;
        }
        sh.a2i[wave_of_lane()][lane] = inc;
    }
    wave_lds_sync();
    float box = 0.0f;
    {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const float v = sh.a2s[wave_of_lane()][d >> 4][gbase + (d & 15)];
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
        const int dn = half ? C::H : D;  // features the A1 bounds cover
        const float qs = l < dn ? q[l] : 0.0f;
        const float qs2 = (D > 16 && l + 16 < dn) ? q[l + 16] : 0.0f;
        const float qn0 = fsum16(__builtin_fmaf(qs2, qs2, __builtin_fmaf(qs, qs, 0.0f)));
        float M = 0.0f;
#pragma unroll
        for (int w = 0; w < NW; ++w) M = fmaxf(M, sh.cnmax[w]);
        const float eps = fadd(fadd(fmul(fadd(qn0, M), C::EPSF), 1e-37f), te);
        const float qn = fadd(qn0, twh);  // the tail's midpoint (0 in full-dimension passes)
#ifndef GSC_NO_LEAF_EPS
        // Per-leaf error bounds.  The A1 value of a leaf c is within
        // (|q|^2 + |c|^2) EPSF (+ TE) of the reference's distance -- the
        // analysis above bounds every rounding by the leaf's own norms; M only
        // stands in for |c|^2 -- and |c|^2 <= 2|q|^2 + 2|q - c|^2 with
        // |q - c|^2 <= qn0 + v + 2 eg (v = the leaf's A1 value, eg = the
        // frame-wide bound without TE; the factor 1 + 2^-20 covers this
        // arithmetic).  So a leaf with A1 value v errs by at most epsv(v), and
        // v - epsv(v) grows with v: bounds that hold for a subtree's minimum
        // hold for all its leaves.  A quiet query among loud centroids (|q|^2,
        // |q - c|^2 << M) gets its own scale instead of the loudest centroid's.
        const float eg = fmul(fadd(qn0, M), C::EPSF);
        auto epsv = [&](uint32_t vb) {
            const float v = __uint_as_float(vb);
            const float dq = fmaxf(fadd(fadd(qn0, v), fadd(eg, eg)), 0.0f);
            const float cb = fmul(fadd(fadd(qn0, qn0), fadd(dq, dq)), 1.0f + 0x1p-20f);
            return fadd(fadd(fmul(fadd(qn0, fminf(cb, M)), C::EPSF), 1e-37f), te);
        };
        const float es = epsv(gmin), e2 = epsv(m2), eb = epsv(sib);
        ok = !far || (fsub(fadd(qn, __uint_as_float(sib)), eb) > Bv);
        unique = fsub(__uint_as_float(m2), __uint_as_float(gmin)) > fadd(es, e2);
        m2lo = fsub(fadd(qn, __uint_as_float(m2)), e2);
#else
        ok = !far || (fsub(fadd(qn, __uint_as_float(sib)), eps) > Bv);
        unique = fsub(__uint_as_float(m2), __uint_as_float(gmin)) > fadd(eps, eps);
        m2lo = fsub(fadd(qn, __uint_as_float(m2)), eps);
#endif
        const bool gfail = !unique || ((__ballot(!ok) >> gbase) & 0xFFFFull) != 0;
#ifdef GSC_STAMPS
        if (xc) xc[9] += __popcll(__ballot(gfail && l == 0 && qa));  // queries needing the per-wave bounds
#endif
        if (__ballot(gfail) != 0) {
            // a query of this wave failed with the frame-wide bound: retry with an
            // error bound per wave.  A leaf of wave w has |c|^2 <= cnmax[w]
            // (monotone within the pass, so it covers any earlier snapshot), so its
            // A1 value is within eps_w = (|q|^2 + cnmax[w]) EPSF (+ TE) of the
            // reference's distance: quiet queries among quiet centroids get their
            // own scale instead of the frame's loudest centroid's
            auto epsw = [&](int w) { return fadd(fadd(fmul(fadd(qn0, sh.cnmax[w]), C::EPSF), 1e-37f), te); };
            const float eW = epsw(Wv);
            float eS = eW;  // the sibling subtree's bound: its waves' (wave-level depths) or W's
            if (l < KW) {
                const int sh_ = KW - 1 - l;
                const int want = (W >> sh_) ^ 1;
                eS = 0.0f;
#pragma unroll
                for (int w = 0; w < NW; ++w)
                    if ((w >> sh_) == want) eS = fmaxf(eS, epsw(w));
            }
            ok = !far || (fsub(fadd(qn, __uint_as_float(sib)), eS) > Bv);
            // c* beats every other leaf: W's own other leaves (lane / slot depths)
            // and every other wave's minimum, each with its wave's bound
            const float gm = __uint_as_float(gmin);
            const float m2W = __uint_as_float(fmin16((l >= KW && l < LOGK) ? sib : kInfBits));
            const bool ow = l < NW && l != Wv;  // lane l: another wave's record
            const float el = ow ? epsw(l) : 0.0f;
            const bool uw = !ow || fsub(__uint_as_float(mw), gm) > fadd(eW, el);
            unique = fsub(m2W, gm) > fadd(eW, eW) && ((__ballot(!uw) >> gbase) & 0xFFFFull) == 0;
            const float lo_l = ow ? fsub(fadd(qn, __uint_as_float(mw)), el) : __builtin_inff();
            m2lo = fminf(fsub(fadd(qn, m2W), eW), __uint_as_float(fmin16(__float_as_uint(lo_l))));
        }
    } else {
        ok = !far || (__uint_as_float(sib) > Bv);
        unique = !tie;
        m2lo = __uint_as_float(m2);
    }
    if (far && inc != inc) ok = false;  // a NaN box' is never visited (fmaxf would drop it from B)
    const bool gok = ((__ballot(!ok) >> gbase) & 0xFFFFull) == 0;
    const bool valid = unique && __uint_as_float(gmin) <= FLT_MAX && gok;
#ifdef GSC_STAMPS
    if (xc && APPROX) {  // why approximate certificates fail: no unique minimum / a far step not provable
        xc[10] += __popcll(__ballot(qa && l == 0 && !unique));
        xc[11] += __popcll(__ballot(qa && l == 0 && unique && !gok));
    }
#endif
    // NaN centroids (their leaves carry +inf in every distance here): ANN's DFS
    // reaches first the leaf of the near-child descent; a NaN leaf there becomes
    // the answer with key NaN (every later box' < NaN test fails) -- otherwise
    // NaN leaves are inert (key > NaN is false), which the +inf distances model.
    // The descent equals c*'s root path when no step of it is far.
    int nanf = -1;
    if (APPROX && nanpass && qa && l == 0 && farmask != 0) {
        int h = 0, pos = 0;
#pragma unroll 1
        for (int lv = 0; lv < LOGK; ++lv) {
            const int bit = fsub(q[sh.t.cd[h]], sh.t.cv[h]) < 0.0f ? 0 : 1;
            pos = 2 * pos + bit;
            h = 2 * h + 1 + bit;
        }
        const int id = sh.t.pidx[pos];
        if (id != 0xFFFF && ((sh.nanid[id >> 5] >> (id & 31)) & 1u)) nanf = pos;
    }
    if (qa) {
        QRecT<D>& R = recs[jj];
        if (l < LOGK) R.B[l] = Bv;
        if (l == 0) {
            const int cs = nanf >= 0 ? nanf : cstar;
            R.valid = (valid || nanf >= 0) ? 1 : 0;
            R.cstar = cs;
            R.id = sh.t.pidx[cs];
            R.g = nanf >= 0 ? __builtin_nanf("") : __uint_as_float(gmin);  // exact mode only (the solo query); batch queries: vp_end
            R.m2 = m2lo;
            R.rate = sh.rate[cs];
            R.farmask = farmask;
            R.pad_ = nanf >= 0 ? 1 : 0;  // NaN-first query: no move, no check, residual NaN
        }
    }
    ASTAMP(15)
    (void)LS;
}
#undef ASTAMP

// ---------------------------------------------------------------------------
// Commit, step 1 (wave 0, lanes = queries j of the pending batch): online
// updates in order per centroid (encoder.lpr:735-740, f32 c += (x - c) * rate)
// assuming every query of the batch commits; version table for the checks.
// Log entry e is lane e: position lg_pos (-1 = empty), tag = commit iteration.
// ---------------------------------------------------------------------------
// Scan state of one pending query (lane j) / log entry (lane e).
struct VPState {
    int cs, pred, nxt, first, ie;
};

template <class C>
__device__ __forceinline__ void vp_begin(Scan2Shared<C>& sh, int qb, int off, int pn, int a1, int lane, int& lg_pos,
                                         int lg_tag, VPState& st) {
    if (lg_pos >= 0 && lg_tag < a1) lg_pos = -1;  // committed before the batch's snapshot
    // a NaN-first query moves nothing: a key of its own, so it joins no chain and no log entry
    st.cs = lane < pn ? (sh.qrec[qb][off + lane].pad_ ? -100 - lane : sh.qrec[qb][off + lane].cstar) : -2;
    sh.vmeta[lane].x = lg_pos;
    sh.vmeta[lane].y = 0;
    if (lane < C::KB) sh.vcs[lane] = st.cs;
    // pairs (query, query with the same c*) and (log entry, query moving it) by
    // position masks in LDS: qm[p] = the batch's queries whose c* is leaf p.
    // dfs_inc is free here (the exact DFS runs in part 4, behind barriers) and
    // only this wave touches it now; positions are unique among log entries
    uint32_t* qm = reinterpret_cast<uint32_t*>(sh.dfs_inc);
    const int cs = st.cs;
    const bool qv = lane < C::KB && cs >= 0;
    if (qv) qm[cs] = 0u;
    if (lg_pos >= 0) qm[lg_pos] = 0u;
    if (lane < C::KB) sh.vie[lane] = 64;
    wave_lds_sync();
    if (qv) atomicOr(&qm[cs], 1u << lane);
    wave_lds_sync();
    const uint32_t mq = qv ? qm[cs] : 0u;               // queries sharing c*_j
    const uint32_t me = lg_pos >= 0 ? qm[lg_pos] : 0u;  // queries moving entry e's centroid
    const uint32_t below = lane < 32 ? (1u << lane) - 1u : ~0u;
    const uint32_t above = lane < 31 ? ~((2u << lane) - 1u) : 0u;
    const uint32_t mb = mq & below, ma = mq & above;
    st.pred = mb ? 64 + (31 - __clz(mb)) : -1;   // last earlier query with the same c*
    st.nxt = ma ? __ffs(ma) - 1 : C::KB;          // first later one
    st.first = me ? __ffs(me) - 1 : C::KB;        // lane as log entry: first query moving it
    for (uint32_t m = me; m; m &= m - 1u) atomicMin(&sh.vie[__ffs(m) - 1], lane);  // the entry holding c*_j
    wave_lds_sync();
    st.ie = lane < C::KB ? sh.vie[lane] : 64;
}

template <class C>
__device__ __forceinline__ void vp_end(Scan2Shared<C>& sh, int qb, int off, int pn, int lane, int lg_pos,
                                       const VPState& st, bool half, int par) {
    constexpr int D = C::D, KB = C::KB;
    const int j = lane;
    const bool act = j < pn;
    const QRecT<D>& R = sh.qrec[qb][off + (act ? j : 0)];
    const int cs = st.cs, nxt = st.nxt;
    const int ie = st.ie < 64 ? st.ie : -1;  // log entry holding c*_j (c*_j moved before the batch)
    const int pred = st.pred >= 0 ? st.pred : ie;
    // versions: log entries (0..63) and "after query j" (64+j)
    sh.vmeta[lane].z = lg_pos >= 0 ? st.first : -1;
    if (lane < KB) {
        sh.vmeta[64 + lane] = make_int4(act ? cs : -1, j + 1, act ? nxt : -1, 0);
        sh.nxt[par][lane] = nxt;
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
            const float* o = pred < 0 ? R.o : (pred < 64 ? sh.lg_c[pred] : sh.newc[par][pred - 64]);
            float oc[D];
#pragma unroll
            for (int d = 0; d < D; ++d) oc[d] = o[d];
            // exact live distance to c* (its snapshot coordinates when unmoved;
            // the A1 values of the batch are bounds only)
            const bool nanq = R.pad_ != 0;
            const float gpj = nanq ? __builtin_nanf("") : seqdist<D>(qv, oc);
            const bool okc = nanq || (R.valid != 0 && (pred < 0 || gpj < R.m2));
            const float rate = R.rate;
            float nrm = 0.0f;  // |new c|^2 over the features the A1 bounds cover (norm2_x's order)
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const float nc = fadd(oc[d], fmul(fsub(qv[d], oc[d]), rate));
                sh.newc[par][j][d] = nc;
                if (d < C::H || !half) nrm = __builtin_fmaf(nc, nc, nrm);
            }
            sh.newc[par][j][C::ROW - 1] = nrm;
            sh.gp[j] = gpj;
#ifdef GSC_STAMPS
            if (!okc) sh.inval[j] = R.valid == 0 ? 1 : (R.valid == 2 ? 8 : 2);  // cause (stamps): uncertified / c* moved past m2 (DFS answer: away)
#else
            if (!okc) sh.inval[j] = 1;
#endif
        }
        wave_lds_sync();  // this round's newc feed the next round's lanes
        done |= rm;
    }
}

// A centroid at kd-leaf vp, moved since the snapshot to live distance du, and
// the snapshot DFS answer of R (valid == 2; g = c*'s live distance): ANN's
// improvement sequence -- and so its answer -- is unchanged when du is not
// below the best-so-far at vp's DFS rank (ann_search inserts only strictly
// smaller distances), vp was not an improvement itself, and c* did not move
// away (vp_end).  The best-so-far at vp's rank is the distance of the last
// improvement that ranks before vp; vp ranks after leaf p iff p's root path
// takes the near child at the split where the two paths part, i.e. p's rank
// (whose bit LOGK-1-l is the far step at depth l) has a 0 there.  Leaves the
// DFS prunes need no case of their own: a leaf that is no improvement when
// reached changes nothing whether or not it is reached.
template <int LOGK, int D>
__device__ __forceinline__ bool dfs_keeps(const QRecT<D>& R, float du, int vp, float g) {
    const int n = R.nimp;
#pragma unroll 1
    for (int i = n - 1; i >= 0; --i) {
        const int x = R.ir[i];
        const int pos = x & 4095, rk = x >> 12;
        if (vp == pos) return false;  // an earlier improvement moved (vp is never c* here)
        const int l = __clz((uint32_t)(vp ^ pos)) - (32 - LOGK);
        if (((rk >> (LOGK - 1 - l)) & 1) == 0) return !(du < (i == n - 1 ? g : R.B[i]));
    }
    return false;  // vp ranks before the first leaf reached: impossible (rank 0), kept conservative
}

// The same checks as work items taken by whichever wave is free (one-CU
// frames).  A1 is uneven across waves -- pruning leaves some waves a third of
// the queries of others -- so the waves that finish A1 first run the V check
// while the others still compute distances, instead of every wave doing an
// eighth of it after the A1 barrier.  A trip = two versions per lane group
// (lane = query, two versions per lane group); the next trip's index is taken at the start of a trip
// (LDS atomic), and the checks start once wave 0's update chain (vp_end) of
// this iteration is published (vp_ready).
template <class C>
__device__ __forceinline__ void v_check_grab(Scan2Shared<C>& sh, int qb, int off, int pn, int lane, int par) {
    constexpr int D = C::D, KB = C::KB, QPL = 64 / KB, LOGK = C::LOGK;
    constexpr int VPT = 2 * QPL;  // versions per trip
    constexpr int NTRIP = (C::KVER + VPT - 1) / VPT;
    int t = 0;
    if (lane == 0) t = atomicAdd(&sh.vc_next, 1);
    t = __builtin_amdgcn_readfirstlane(t);
    if (t >= NTRIP) return;
    const int j = lane % KB, grp = lane / KB;
    const int jr = j < pn ? j : 0;
    const QRecT<D>& R = sh.qrec[qb][off + jr];
    const bool act = j < pn && R.pad_ == 0;  // a NaN-first answer holds whatever moved
    const bool dfsa = R.valid == 2;          // the snapshot DFS answer (dfs_keeps)
    const int cs = R.cstar;
    const uint32_t fm = R.farmask;
    const float g = sh.gp[jr];
    float q[D];
#pragma unroll
    for (int d = 0; d < D; ++d) q[d] = sh.q[qb][off + jr][d];
    bool bad = false;
#pragma unroll 1
    while (t < NTRIP) {
        int tn = 0;
        if (lane == 0) tn = atomicAdd(&sh.vc_next, 1);  // the next trip, in flight during this one
        const int v0 = t * VPT + 2 * grp;
        const bool h0 = v0 < C::KVER, h1 = v0 + 1 < C::KVER;
        const int v0s = h0 ? v0 : 0, v1 = h1 ? v0 + 1 : v0s;
        // the metadata of both versions in one LDS round trip (no short-circuit
        // branches between dependent reads)
        const int4 m0 = sh.vmeta[v0s], m1 = sh.vmeta[v1];
        const int vp0 = h0 ? m0.x : -1, vp1 = h1 ? m1.x : -1;
        const bool u0 = (vp0 >= 0) & act & (j >= m0.y) & (j <= m0.z) & (vp0 != cs);
        const bool u1 = (vp1 >= 0) & act & (j >= m1.y) & (j <= m1.z) & (vp1 != cs);
        if (u0 || u1) {
            const float* c0 = v0s < 64 ? sh.lg_c[v0s] : sh.newc[par][v0s - 64];
            const float* c1 = v1 < 64 ? sh.lg_c[v1] : sh.newc[par][v1 - 64];
            const int lca0 = __clz(vp0 ^ cs) - (32 - LOGK), lca1 = __clz(vp1 ^ cs) - (32 - LOGK);
            const float b0 = R.B[lca0 & 15], b1 = R.B[lca1 & 15];
            float du0 = 0.0f, du1 = 0.0f;
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const float t0 = fsub(q[d], c0[d]), t1 = fsub(q[d], c1[d]);
                du0 = fadd(du0, fmul(t0, t0));
                du1 = fadd(du1, fmul(t1, t1));
            }
            const bool far0 = (fm >> (lca0 & 31)) & 1u, far1 = (fm >> (lca1 & 31)) & 1u;
            if (!dfsa) {
                if (u0 && !(du0 > g && (!far0 || du0 > b0))) bad = true;
                if (u1 && !(du1 > g && (!far1 || du1 > b1))) bad = true;
            } else {
                if (u0 && !dfs_keeps<LOGK, D>(R, du0, vp0, g)) bad = true;
                if (u1 && !dfs_keeps<LOGK, D>(R, du1, vp1, g)) bad = true;
            }
        }
        t = __builtin_amdgcn_readfirstlane(tn);
    }
#ifdef GSC_STAMPS
    if (bad) atomicOr(&sh.inval[j], 4);  // cause (stamps): a moved centroid broke the certificate
#else
    if (bad) sh.inval[j] = 1;
#endif
}

// Exact ANN ann_search (k = 1, eps = 0; annkSearch @0x1800124b0), all
// threads: the result of the stale-tree DFS is decided by its strict
// improvements only.  With leaves ranked in near-first DFS order, a leaf is
// reached while the best distance is b iff every far subtree on its path
// entered after the current best was found has box' < b; box' only grows
// along a path, so that is one test on its innermost far subtree (start rank
// s*, box' bx*).  The next improvement is the lowest-ranked reached leaf with
// d < b, found by one block min-reduction per improvement.  Live leaf
// distances come from sh.dist.  Passes with NaN centroids do not come here:
// their trees can have cells whose bounds contradict the cut values (NaN cuts
// upstream), so box' can shrink along a path (negative increments) and the
// innermost-far-subtree test is not enough; they run scan_exact_dfs.
//
// With `rec` the improvements (DFS rank, leaf, distance) go to rec->ir / B /
// nimp (thread 0): the in-batch DFS answers' validity check (v_check_grab)
// replays the rank order of a moved centroid against them.
template <class C>
__device__ __forceinline__ void dfs_parallel(Scan2Shared<C>& sh, const float* __restrict__ q, int tid, int lane,
                                             int wave, int& out_pos, float& out_key, QRecT<C::D>* rec = nullptr) {
    constexpr int D = C::D, LOGK = C::LOGK, NW = C::NWL;
    constexpr int K = 1 << LOGK;
    constexpr int nthreads = 64 * NW;
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
    // this thread's 8 leaves (an aligned depth LOGK-3 subtree): DFS rank, start
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
    int pos = -1, bp = -1, par = 0, nimp = 0;
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
        if (rec && tid == 0 && nimp < kMaxImp) {
            rec->ir[nimp] = (int)g;
            rec->B[nimp] = b;
        }
        ++nimp;
    }
    if (rec && tid == 0) rec->nimp = nimp;
    out_pos = bp;
    out_key = b;
}

// the exact DFS as a call: at D = 8 the inlined DFS's registers cost the
// kernel 20 spilled VGPRs elsewhere and the call costs nothing measurable
// (C5 -cs4 6336 vs 6335 ms); at D = 16 the inlined DFS is 0.4 % faster
template <class C>
__device__ __noinline__ void dfs_parallel_call(Scan2Shared<C>& sh, const float* __restrict__ q, int tid, int lane,
                                               int wave, int& out_pos, float& out_key, QRecT<C::D>* rec) {
    dfs_parallel<C>(sh, q, tid, lane, wave, out_pos, out_key, rec);
}

// Exact ANN search of the NaN passes, all threads.  NaN cut values and the
// cells below them (bounds that contradict the cuts) make box' increments of
// any sign, or NaN, so box' need not grow along a path and dfs_parallel's
// one test on the innermost far subtree is not enough.  The rank argument
// still holds: with the current best b found at DFS rank pos, a later leaf is
// reached before the next improvement iff every far subtree on its path that
// STARTS after pos has box' < b -- those are tested with b, the ones starting
// before pos contain pos and were entered -- and starts grow with depth, so
// that is a suffix of the path's far steps.  Each improvement round walks the
// paths of the thread's 8 leaves (the first LOGK-3 levels shared) and takes
// the suffix maximum of box' (NaN = +inf: never entered, ANN's `box' < key`
// is false); the next improvement is the lowest-ranked reached leaf with
// d < b (one block min-reduction per improvement, as in dfs_parallel).  NaN
// and dead leaves carry +inf in sh.dist and never improve.  Same answers as
// ANN's sequential walk (annkSearch @0x1800124b0; the oracle's ann_oracle.c).
template <class C>
__device__ __noinline__ void dfs_parallel_nan(Scan2Shared<C>& sh, const float* __restrict__ q, int tid, int lane,
                                                 int wave, int& out_pos, float& out_key, QRecT<C::D>* rec) {
    constexpr int D = C::D, LOGK = C::LOGK, NW = C::NWL;
    constexpr int K = 1 << LOGK;
    constexpr int nthreads = 64 * NW;
    for (int h0 = 0; h0 < K; h0 += nthreads) {  // split nodes: signed box' increment, near child
        const int h = h0 + tid;
        bool nearlo = false;
        if (h < K - 1) {
            const float qc = q[sh.t.cd[h]];
            const float cut = fsub(qc, sh.t.cv[h]);
            nearlo = cut < 0.0f;
            float bd = nearlo ? fsub(sh.t.lo[h], qc) : fsub(qc, sh.t.hi[h]);
            if (bd < 0.0f) bd = 0.0f;
            sh.dfs_inc[h] = fsub(fmul(cut, cut), fmul(bd, bd));  // any sign, or NaN
        }
        const uint64_t m = __ballot(nearlo);  // 64 consecutive nodes per wave
        if (lane == 0) {
            sh.dfs_near[(h0 + wave * 64) >> 5] = (uint32_t)m;
            sh.dfs_near[((h0 + wave * 64) >> 5) + 1] = (uint32_t)(m >> 32);
        }
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
    // The paths do not depend on the improvement round, only the choice of
    // far steps does: with the leaf's DFS rank R > pos and t the highest bit
    // where R and pos differ, the far steps with start > pos are exactly those
    // at levels >= LOGK - 1 - t.  So each path is walked once, keeping the
    // suffix maxima of box' by level (NaN = +inf): shared over the thread's
    // top LOGK - 3 levels, per leaf over the last three.
    const int p0 = tid * 8;
    constexpr int LT = LOGK - 3;  // shared levels
    float smt[LT + 1];            // suffix max of the shared far boxes from level l
    int preft = 0;                // rank prefix of the thread's 8 leaves
    float boxt = rootbox;
    int ht = 0;
    {
        float fb[LT];
#pragma unroll
        for (int l = 0; l < LT; ++l) {
            const int bit = (p0 >> (LOGK - 1 - l)) & 1;
            const int nearbit = ((sh.dfs_near[ht >> 5] >> (ht & 31)) & 1u) ? 0 : 1;
            fb[l] = -__builtin_inff();
            if (bit != nearbit) {  // the leaf lies in the far child: its subtree starts after the near one
                boxt = fadd(boxt, sh.dfs_inc[ht]);
                preft += 1 << (LOGK - 1 - l);
                fb[l] = boxt != boxt ? __builtin_inff() : boxt;
            }
            ht = 2 * ht + 1 + bit;
        }
        smt[LT] = -__builtin_inff();
#pragma unroll
        for (int l = LT - 1; l >= 0; --l) smt[l] = fmaxf(fb[l], smt[l + 1]);
    }
    int rk[8];        // the leaves' DFS ranks
    float sb[8][3];   // per leaf: suffix max of its own far boxes from level LT + j
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {
        float box = boxt, fb[3];
        int pref = preft, h = ht;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int l = LT + j;
            const int bit = ((p0 + s8) >> (LOGK - 1 - l)) & 1;
            const int nearbit = ((sh.dfs_near[h >> 5] >> (h & 31)) & 1u) ? 0 : 1;
            fb[j] = -__builtin_inff();
            if (bit != nearbit) {
                box = fadd(box, sh.dfs_inc[h]);
                pref += 1 << (LOGK - 1 - l);
                fb[j] = box != box ? __builtin_inff() : box;
            }
            h = 2 * h + 1 + bit;
        }
        rk[s8] = pref;
        sb[s8][2] = fb[2];
        sb[s8][1] = fmaxf(fb[1], fb[2]);
        sb[s8][0] = fmaxf(fb[0], sb[s8][1]);
    }
    int pos = -1, bp = -1, par = 0, nimp = 0;
    float b = FLT_MAX;  // the empty list's max_key
    for (;;) {
        uint32_t key = 0xFFFFFFFFu;
        const int gt = preft >> 3, gp = pos >> 3;  // (pos = -1: gp = -1)
        if (gt > gp) {  // every leaf of the thread ranks after pos; t >= 3
            const int t = 31 - __builtin_clz((uint32_t)(preft ^ pos));
            const int lt = max(0, LOGK - 1 - t);
            float mt = smt[0];
#pragma unroll
            for (int l = 1; l < LT; ++l) mt = l == lt ? smt[l] : mt;
#pragma unroll
            for (int s8 = 0; s8 < 8; ++s8) {
                const float M = fmaxf(mt, sb[s8][0]);
                if (p0 + s8 < K && M < b && sh.dist[p0 + s8] < b)
                    key = min(key, ((uint32_t)rk[s8] << 12) | (uint32_t)(p0 + s8));
            }
        } else if (gt == gp) {  // pos inside the thread's group: only the last three levels choose
#pragma unroll
            for (int s8 = 0; s8 < 8; ++s8) {
                const int x = (rk[s8] ^ pos) & 7;
                if (rk[s8] > pos && x != 0) {
                    const int t = 31 - __builtin_clz((uint32_t)x);  // 0..2
                    const float M = t == 2 ? sb[s8][0] : (t == 1 ? sb[s8][1] : sb[s8][2]);
                    if (p0 + s8 < K && M < b && sh.dist[p0 + s8] < b)
                        key = min(key, ((uint32_t)rk[s8] << 12) | (uint32_t)(p0 + s8));
                }
            }
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
        if (rec && tid == 0 && nimp < kMaxImp) {  // the improvement sequence (as dfs_parallel)
            rec->ir[nimp] = (int)g;
            rec->B[nimp] = b;
        }
        ++nimp;
    }
    if (rec && tid == 0) rec->nimp = nimp;
    out_pos = bp;
    out_key = b;
}

// fold published log entries into the owners' registers: two entries per
// trip (both rows read before either is applied), the pruning box and the
// norm bound accumulated in registers and written once
template <class C>
__device__ __forceinline__ void refresh(Scan2Shared<C>& sh, float (&creg)[C::SL][C::DR], float (&cn)[C::SL],
                                        float& cnmax, int vwave, int lane, float* __restrict__ trow = nullptr) {
    constexpr int SL = C::SL, LS = C::LS, D = C::D, DR = C::DR;
    const int pp = sh.pub_pos[lane];
    uint64_t m = __ballot(pp >= 0 && (pp >> (6 + LS)) == vwave);
    if (!m) return;
    float blo = __builtin_inff(), bhi = -__builtin_inff();  // lane d < D: the new positions' range
    auto apply = [&](int e, int p, const float* r, float nv) {
        const int owner = (p >> LS) & 63, slot = p & (SL - 1);
#pragma unroll
        for (int s = 0; s < SL; ++s) {
            if (s == slot) {
#pragma unroll
                for (int d = 0; d < DR; ++d) creg[s][d] = lane == owner ? r[d] : creg[s][d];
                cn[s] = lane == owner ? nv : cn[s];
            }
        }
        if constexpr (C::SPLIT) {  // the owner's tail row (only the owner lane ever reads it)
            if (lane == owner)
                for (int d = DR; d < D; ++d) trow[(int64_t)p * C::TL + (d - DR)] = sh.lg_c[e][d];
        }
    };
    // two entries per trip where the second row fits the register budget (D = 8;
    // at D = 16 the extra 16 VGPRs cost 40 spilled registers elsewhere)
    constexpr bool PAIR = DR <= 8;
    while (m) {
        const int e0 = __ffsll((long long)m) - 1;
        m &= m - 1;
        const bool two = PAIR && m != 0;
        const int e1 = two ? __ffsll((long long)m) - 1 : e0;
        if (two) m &= m - 1;
        const int p0 = __builtin_amdgcn_readlane(pp, e0), p1 = __builtin_amdgcn_readlane(pp, e1);
        float r0[DR], r1[PAIR ? DR : 1];
#pragma unroll
        for (int d = 0; d < DR; ++d) {
            r0[d] = sh.lg_c[e0][d];
            if constexpr (PAIR) r1[d] = sh.lg_c[e1][d];
        }
        const float nv0 = sh.lg_c[e0][C::ROW - 1], nv1 = sh.lg_c[e1][C::ROW - 1];  // |c|^2, written with the entry
        if (lane < D) {  // the pruning box covers the new positions
            const float v0 = sh.lg_c[e0][lane], v1 = sh.lg_c[e1][lane];
            blo = fminf(blo, fminf(v0, v1));
            bhi = fmaxf(bhi, fmaxf(v0, v1));
        }
        // the wave's norm bound only grows within a pass (A2 reads it for any earlier snapshot)
        cnmax = fmaxf(cnmax, fmaxf(nv0, nv1));
        apply(e0, p0, r0, nv0);
        if constexpr (PAIR) {
            if (two) apply(e1, p1, r1, nv1);
        }
    }
    if (lane < D) {
        sh.wlo[vwave][lane] = fminf(sh.wlo[vwave][lane], blo);
        sh.whi[vwave][lane] = fmaxf(sh.whi[vwave][lane], bhi);
    }
    if (lane == 0) sh.cnmax[vwave] = cnmax;
}

// fold the pending batch's committed updates (its first kc queries) into the
// owners' registers, straight from the update chain's rows: query j carries
// the last committed update of its c* when no later committed query of the
// batch shares c* (the commit logs the same row, part 3)
template <class C>
__device__ __forceinline__ void fold_commits(Scan2Shared<C>& sh, float (&creg)[C::SL][C::DR], float (&cn)[C::SL],
                                             float& cnmax, int vwave, int lane, int qb, int off, int kc, int par,
                                             float* __restrict__ trow = nullptr) {
    constexpr int SL = C::SL, LS = C::LS, D = C::D, DR = C::DR;
    int pp = 0;
    bool mine = false;
    if (lane < kc) {
        const QRecT<D>& R = sh.qrec[qb][off + lane];
        pp = R.cstar;
        mine = sh.nxt[par][lane] >= kc && R.pad_ == 0 && (pp >> (6 + LS)) == vwave;
    }
    uint64_t m = __ballot(mine);
    if (!m) return;
    float blo = __builtin_inff(), bhi = -__builtin_inff();  // lane d < D: the new positions' range
    auto apply = [&](int e, int p, const float* r, float nv) {
        const int owner = (p >> LS) & 63, slot = p & (SL - 1);
#pragma unroll
        for (int s = 0; s < SL; ++s) {
            if (s == slot) {
#pragma unroll
                for (int d = 0; d < DR; ++d) creg[s][d] = lane == owner ? r[d] : creg[s][d];
                cn[s] = lane == owner ? nv : cn[s];
            }
        }
        if constexpr (C::SPLIT) {  // the owner's tail row (only the owner lane ever reads it)
            if (lane == owner)
                for (int d = DR; d < D; ++d) trow[(int64_t)p * C::TL + (d - DR)] = sh.newc[par][e][d];
        }
    };
    // two rows per trip where the second fits the register budget (as refresh)
    constexpr bool PAIR = DR <= 8;
    while (m) {
        const int e0 = __ffsll((long long)m) - 1;
        m &= m - 1;
        const bool two = PAIR && m != 0;
        const int e1 = two ? __ffsll((long long)m) - 1 : e0;
        if (two) m &= m - 1;
        const int p0 = __builtin_amdgcn_readlane(pp, e0), p1 = __builtin_amdgcn_readlane(pp, e1);
        float r0[DR], r1[PAIR ? DR : 1];
#pragma unroll
        for (int d = 0; d < DR; ++d) {
            r0[d] = sh.newc[par][e0][d];
            if constexpr (PAIR) r1[d] = sh.newc[par][e1][d];
        }
        const float nv0 = sh.newc[par][e0][C::ROW - 1], nv1 = sh.newc[par][e1][C::ROW - 1];  // |c|^2 (vp_end)
        if (lane < D) {  // the pruning box covers the new positions
            const float v0 = sh.newc[par][e0][lane], v1 = sh.newc[par][e1][lane];
            blo = fminf(blo, fminf(v0, v1));
            bhi = fmaxf(bhi, fmaxf(v0, v1));
        }
        cnmax = fmaxf(cnmax, fmaxf(nv0, nv1));  // only grows within a pass
        apply(e0, p0, r0, nv0);
        if constexpr (PAIR) {
            if (two) apply(e1, p1, r1, nv1);
        }
    }
    if (lane < D) {
        sh.wlo[vwave][lane] = fminf(sh.wlo[vwave][lane], blo);
        sh.whi[vwave][lane] = fmaxf(sh.whi[vwave][lane], bhi);
    }
    if (lane == 0) sh.cnmax[vwave] = cnmax;
}

// c*'s snapshot coordinates for the queries in qmask (columns col0 + j),
// written by the lane that owns c* (the first wave / lane / slot at the
// minimum of the A1 records, as in A2) into recs[j].o
template <class C>
__device__ __forceinline__ void write_cstar(Scan2Shared<C>& sh, const float (&creg)[C::SL][C::DR], QRecT<C::D>* recs,
                                            uint64_t qmask, int col0, int wave, int lane,
                                            const float* __restrict__ trow = nullptr) {
    constexpr int SL = C::SL, D = C::D, NWL = C::NWL;
    // lane = query: the winning wave (first at the minimum) and, for this
    // wave's wins, the owner lane and slot from its record -- all queries at
    // once, so the copy loop below has no LDS round trip per query
    uint64_t won;
    int ol = 0;  // owner lane << 8 | slot
    {
        const bool act = (qmask >> lane) & 1ull;
        const int jq = act ? lane : 0;
        float gm = __builtin_inff();
        int W = 0;
#pragma unroll
        for (int w = 0; w < NWL; ++w) {
            const float m = __uint_as_float(sh.wrec[w][col0 + jq].minbits);
            if (m < gm) {
                gm = m;
                W = w;
            }
        }
        won = __ballot(act && W == wave);
        if (act && W == wave) {
            const WaveRecT<SL>& r = sh.wrec[wave][col0 + jq];
            bool tie2;
            const int slot = rec_slot<SL>(r, &tie2);
            ol = ((r.lanebits & 255) << 8) | slot;
        }
    }
    while (won) {
        const int jj = __ffsll((long long)won) - 1;
        won &= won - 1;
        const int o = __builtin_amdgcn_readlane(ol, jj);
        const int owner = o >> 8, slot = o & 255;
        float* dst = recs[jj].o;
#pragma unroll
        for (int s = 0; s < SL; ++s)
            if (s == slot && lane == owner) {
#pragma unroll
                for (int d = 0; d < C::DR; ++d) dst[d] = creg[s][d];
                if constexpr (C::SPLIT) {
                    const float* tr = trow + (int64_t)((wave * 64 + owner) * SL + s) * C::TL;
                    for (int d = C::DR; d < D; ++d) dst[d] = tr[d - C::DR];
                }
            }
    }
}

// ---------------------------------------------------------------------------
// The kernel: one workgroup per frame (blockIdx.x = frame).
// ---------------------------------------------------------------------------
template <class C>
__global__ __launch_bounds__(C::NT) void scan_batch_kernel(ReduceFrame* __restrict__ frames, int nframes,
                                                           const float* __restrict__ Xall, float* __restrict__ Call,
                                                           int* __restrict__ i_scratch,
                                                           const float* __restrict__ rate_tab, double tol,
                                                           int max_passes, int opts,
                                                           float* __restrict__ Tall) {
    constexpr int D = C::D, K = C::K, SL = C::SL, LS = C::LS, NWL = C::NWL, KB = C::KB;
    constexpr int kErrWave = NWL > 1 ? 1 : 0;  // residual + cluster ids (wave 0 keeps the log)
    constexpr bool PRUNE = true;               // A1 pruning by wave boxes
    // uncertified queries of a batch resolved in the batch by the exact DFS on the
    // snapshot (see the fixups below); GSC_INBATCH_DFS_D: the widest D that does it
    constexpr bool kInBatchDfs = D <= GSC_INBATCH_DFS_D;
    const bool no_half = (opts & 1) != 0;      // diagnostic: full-dimension A1 bounds in every pass
    const bool no_prune = (opts & 2) != 0;     // experiment: every wave evaluates every query (no mid-A1 barrier)
    // experiment (opts bits 8..15): queries per speculative batch below KB
    const int kbe = ((opts >> 8) & 255) > 0 && ((opts >> 8) & 255) < KB ? ((opts >> 8) & 255) : KB;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Scan2Shared<C>& sh = *reinterpret_cast<Scan2Shared<C>*>(smem);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int nthreads = C::NT;
    const int vwave = wave;
    const int fi0 = blockIdx.x, fstep = nframes;
    for (int fi = fi0; fi < nframes; fi += fstep) {
    ReduceFrame* frp = frames + fi;
    if (uniform_int(frp->done) || uniform_int(frp->generic)) continue;
    const int N = uniform_int(frp->N);
    // colCount of the residual (encoder.lpr:743): 2*ChunkSize, below D when the slab pads the features
    const int dcol_i = uniform_int(frp->dcol) > 0 ? uniform_int(frp->dcol) : D;
    // best / colCount: a constant power-of-two divisor (an exact multiply) unless the slab is padded
    auto per_col = [dcol_i](float v) { return dcol_i == D ? v / (float)D : v / (float)dcol_i; };
    // ChunksPerFrame that is not a power of two (the -br cost loop,
    // encoder.lpr:1337-1351): ANN's tree over the Kr centroids, embedded in the
    // K = 2^LOGK leaf layout with padding leaves that are never visited (pad_tree)
    const int Kr = uniform_int(frp->K);
    const bool padded = Kr != K;
    const float* __restrict__ X = Xall + uniform_i64(frp->x_off);
    float* C_ = Call + uniform_i64(frp->c_off);
    int* clusters = i_scratch + uniform_i64(frp->n_off);
    int* prev_cnt = i_scratch + uniform_i64(frp->k_off);  // cnts[not Odd(iter)] by centroid id
    int* cnta = i_scratch + uniform_i64(frp->ka_off);     // cnts[Odd(iter)] by kd-leaf position
    // split layout: the tail features of kd-leaf position p at trow + p * TL
    float* trow = C::SPLIT ? Tall + uniform_i64(frp->t_off) : nullptr;
    double prev_err = uniform_int(frp->iters) == 0 ? 3.4028234663852886e+38 : frp->err;  // err := MaxSingle
    if constexpr (PRUNE) {  // box of the frame's data in the tail features (half-dimension A1 bounds)
        constexpr int NT_ = D - C::H;
        static_assert(nthreads % NT_ == 0, "each thread keeps one tail feature");
        __syncthreads();  // the previous frame's readers are done
        if (tid < D) {
            sh.xtlo[tid] = 0x7FFFFFFF;
            sh.xthi[tid] = (int)0x80000000;
        }
        __syncthreads();
        int klo = 0x7FFFFFFF, khi = (int)0x80000000;
        const int d = C::H + tid % NT_;
        for (int64_t r = tid / NT_; r < N; r += nthreads / NT_) {
            const int k = ordkey(__float_as_uint(X[r * D + d]));
            klo = min(klo, k);
            khi = max(khi, k);
        }
        atomicMin(&sh.xtlo[d], klo);
        atomicMax(&sh.xthi[d], khi);
        __syncthreads();
    }

    // All of the frame's passes run in this launch (the pass index lives in
    // the frame descriptor), so a frame never waits for the slowest frame of a
    // pass; a NaN pass returns and the generic kernel takes that pass over.
    for (int pass = uniform_int(frp->iters); pass < max_passes; ++pass) {
#ifdef GSC_STAMPS
    const uint64_t t_kernel0 = stamp();
#endif
    if (pass == 0)
        for (int k = tid; k < Kr; k += nthreads) prev_cnt[k] = 1;  // CCntStart (encoder.lpr:717-721)
    if (tid == 0) sh.any_nan = 0;
    // NaN rows (yakmo's 0/0 means of seeds that won no point) stay NaN in every
    // pass and finite rows stay finite (c + (x - c) * rate): their leaves carry
    // +inf distances here (inert in ANN's DFS once a real leaf was reached) and
    // the queries whose descent reaches one first take it (a2_group)
    for (int w = tid; w < kMaxK / 32; w += nthreads) sh.nanid[w] = 0u;
    __syncthreads();
    int nan_rows = 0;
    for (int k = tid; k < Kr; k += nthreads) {
        bool nn = false;
#pragma unroll
        for (int d = 0; d < D; ++d) nn |= C_[(int64_t)k * D + d] != C_[(int64_t)k * D + d];
        if (nn) {
            atomicOr(&sh.nanid[k >> 5], 1u << (k & 31));
            nan_rows = 1;
        }
    }
    nan_rows = __syncthreads_or(nan_rows);
    if (padded) {
        build_tree<D>(sh.t, sh.dist, C_, Kr);  // ANN's n/2 splits over the real centroids
        pad_tree<C::LOGK>(sh.t, reinterpret_cast<int*>(sh.dist), Kr, tid, nthreads);
    } else if (nan_rows) {  // NaN coordinates: annMaxSpread's and quickselect's exact order
        if constexpr (K / nthreads >= 4)
            build_tree_nan<D, C::LOGK, nthreads>(sh.t, sh.dist, sh.dfs_inc, C_);
        else
            build_tree<D>(sh.t, sh.dist, C_, K);
    } else if constexpr (K / nthreads < 4) {
        build_tree<D>(sh.t, sh.dist, C_, K);  // one or two leaves per thread: the sequential build
    } else if (!build_tree_fast<D, C::LOGK, nthreads>(sh.t, sh.dist, sh.dfs_inc, C_, &sh.slow_pos)) {
        build_tree<D>(sh.t, sh.dist, C_, K);  // median ties: quickselect's exact order
        if (tid == 0) frp->tree_exact += 1;
    }

    float creg[SL][C::DR];
    float cn[SL];  // |c|^2 (over the register features) per register leaf (A1 bounds); +inf for padding leaves
    const int p0 = (vwave * 64 + lane) * SL;
    bool nan_here = false;
    uint32_t dmask = 0;  // slots that hold no live centroid (past K, padding, NaN rows, dead leaves): +inf distances
    constexpr int TLA = C::TL > 0 ? C::TL : 1;
    float tlo[TLA], thi[TLA];  // split layout: this lane's tail box
#pragma unroll
    for (int d = 0; d < TLA; ++d) {
        tlo[d] = __builtin_inff();
        thi[d] = -__builtin_inff();
    }
#pragma unroll
    for (int s = 0; s < SL; ++s) {
        const int p = p0 + s;
        const int id = p < K ? (int)sh.t.pidx[p] : 0xFFFF;
        // NaN passes: a split node with a NaN cut value sends every query to
        // its high child first and never enters the low one (box' = NaN), so
        // the leaves below a low child of such a node are dead for the pass
        bool dead = false;
        if (nan_rows && p < K) {
#pragma unroll 1
            for (int l = 0, h = 0; l < C::LOGK; ++l) {
                const int bit = (p >> (C::LOGK - 1 - l)) & 1;
                dead |= bit == 0 && sh.t.cv[h] != sh.t.cv[h];
                h = 2 * h + 1 + bit;
            }
        }
        if (id != 0xFFFF && !dead && !((sh.nanid[id >> 5] >> (id & 31)) & 1u)) {
#pragma unroll
            for (int d = 0; d < C::DR; ++d) {
                creg[s][d] = C_[(int64_t)id * D + d];
                nan_here |= creg[s][d] != creg[s][d];
            }
            if constexpr (C::SPLIT) {  // the tail features go to the lane's rows of the tail array
#pragma unroll
                for (int d = 0; d < C::TL; ++d) {
                    const float v = C_[(int64_t)id * D + C::DR + d];
                    trow[(int64_t)p * C::TL + d] = v;
                    nan_here |= v != v;
                    tlo[d] = fminf(tlo[d], v);
                    thi[d] = fmaxf(thi[d], v);
                }
            }
        } else {
            dmask |= 1u << s;
#pragma unroll
            for (int d = 0; d < C::DR; ++d) creg[s][d] = 0.0f;
        }
        cn[s] = (dmask >> s) & 1u ? __builtin_inff() : norm2_x<C::DR>(creg[s]);
    }
    if constexpr (PRUNE) {  // the half-dimension bound's inputs: H-norm maxima, tail box of the centroids
        float mh = 0.0f;
#pragma unroll
        for (int s = 0; s < SL; ++s) mh = fmaxf(mh, (dmask >> s) & 1u ? 0.0f : norm2_x<C::H>(creg[s]));
        mh = wave_max_nonneg(nan_here ? 0.0f : mh);
        if (lane == 0) sh.cnmax_h[vwave] = mh;
#pragma unroll
        for (int d = C::H; d < D; ++d) {
            float lo = __builtin_inff(), hi = -__builtin_inff();
            if constexpr (C::SPLIT) {
                lo = tlo[d - C::H];
                hi = thi[d - C::H];
            } else {
#pragma unroll
                for (int s = 0; s < SL; ++s)
                    if (!((dmask >> s) & 1u)) {
                        lo = fminf(lo, creg[s][d < C::DR ? d : 0]);
                        hi = fmaxf(hi, creg[s][d < C::DR ? d : 0]);
                    }
            }
            const int klo = wave_min_i(ordkey(__float_as_uint(lo)));
            const int khi = wave_max_i(ordkey(__float_as_uint(hi)));
            if (lane == 0) {
                sh.ptlo[vwave][d] = __uint_as_float(keybits(klo));
                sh.pthi[vwave][d] = __uint_as_float(keybits(khi));
            }
        }
    }
    // rates of every position
    for (int p = tid; p < K; p += nthreads) {
        const int id = sh.t.pidx[p];
        sh.rate[p] = id != 0xFFFF ? rate_tab[prev_cnt[id]] : 0.0f;  // Single(1/sqrt(cnts[not Odd(iter)]))
        cnta[p] = 1;
    }
    if (nan_here) sh.any_nan = 1;
    float cnmax;
    {
        float mx = 0.0f;
#pragma unroll
        for (int s = 0; s < SL; ++s) mx = fmaxf(mx, (dmask >> s) & 1u ? 0.0f : cn[s]);
        cnmax = wave_max_nonneg(nan_here ? 0.0f : mx);  // NaN passes leave for the generic kernel below
        if (lane == 0) {
            sh.cnmax[vwave] = cnmax;
            sh.cnmax_f[vwave] = cnmax;
        }
    }
    if constexpr (PRUNE) {
        wave_box_init<C>(sh, creg, vwave, lane, p0, dmask);
        if (tid < KB) sh.ub[tid] = kInfBits;
    }
    if (tid == 0) {  // V check work list: iteration tags start at 1 in every pass
        sh.vc_next = 0;
        sh.vp_ready = 0;
    }
    // first batch's queries
    const int n0 = min(kbe, N);
    for (int k = tid; k < n0 * D; k += nthreads) {
        const float x = X[k];
        sh.q[0][k / D][k % D] = x;
        sh.qm[0][k / D][k % D] = -2.0f * x;
    }
    __syncthreads();
    // half-dimension A1 for this pass?  TW over the box of the frame's data
    // and the pass's centroids (tail features), with an ulp-scale slack per
    // feature for the rounding of the online moves
    bool half = false;
    float twh = 0.0f, te = 0.0f, tw_pass = 0.0f;
    if constexpr (PRUNE) {
        float tw = 0.0f, tn = 0.0f;
#pragma unroll
        for (int d = C::H; d < D; ++d) {
            float lo = __uint_as_float(keybits(sh.xtlo[d])), hi = __uint_as_float(keybits(sh.xthi[d]));
#pragma unroll
            for (int w = 0; w < C::NWV; ++w) {
                lo = fminf(lo, sh.ptlo[w][d]);
                hi = fmaxf(hi, sh.pthi[w][d]);
            }
            const float mag = fmaxf(fabsf(lo), fabsf(hi));
            const float wd = fadd(fsub(hi, lo), fadd(fmul(mag, 0x1p-20f), 1e-30f));
            tw = fadd(tw, fmul(wd, wd));
            tn = fadd(tn, fmul(mag, mag));
        }
        tw = fmul(tw, 1.0f + 0x1p-10f);
        tw_pass = tw;
        float mh = 0.0f;
#pragma unroll
        for (int w = 0; w < C::NWV; ++w) mh = fmaxf(mh, sh.cnmax_h[w]);
        twh = fmul(tw, 0.5f);
        te = fadd(twh, fmul(fmul(fmul(tn, 2.0f), C::EPSF), 1.0f + 0x1p-10f));
        // worth it while the tail slack is a small part of eps's norm scale
        half = !(tw != tw) && te <= fmul(fmul(mh, C::EPSF), 0.25f) && !uniform_int(sh.any_nan) && !no_half;
    }
    if (uniform_int(sh.any_nan) || (C::SPLIT && !half)) {
        // NaN centroids (yakmo 0/0 means) make ANN's early exits order dependent;
        // the split layout has no full-dimension bound (a tail too wide for eps):
        // this pass runs in the generic kernel (gsc_kernels.hip)
        if (tid == 0) frp->generic = 1;
        break;
    }
    if (half) {  // the A1 bounds cover the first H features: H-norms for the bound and for eps's M
#pragma unroll
        for (int s = 0; s < SL; ++s) cn[s] = (dmask >> s) & 1u ? __builtin_inff() : norm2_x<C::H>(creg[s]);
        cnmax = sh.cnmax_h[vwave];
        __syncthreads();  // every wave has read sh.cnmax_h / sh.cnmax above
        if (lane == 0) sh.cnmax[vwave] = cnmax;
        __syncthreads();
    }

    // wave-0 state: update log (lane = entry, tag = commit iteration) + residual (lane 0)
    int lg_pos = -1, lg_tag = 0;
    double err = 0.0;
    int slow_total = 0, restarts = 0;
    // in-batch DFS answers of this pass, and how many failed at the commit: on
    // frames whose answers rarely survive (quiet audio among NaN centroids:
    // 2 in 3 fail on the corpus' 60.wav) the DFS would be paid twice, so the
    // pass stops using it once a third of them fail (uniform counters)
    int ib_try = 0, ib_fail = 0;
    bool guard = false;  // the progress guard tripped
#ifdef GSC_STAMPS
    uint64_t acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t acn[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // home, pruned, evaluated, iterations, fixups, pending
    // wave 0: bubble iterations / cycles, other iterations / cycles, iterations with fixups / cycles,
    // iterations with a solo resolution / cycles, new queries, A2 queries needing per-wave bounds
    uint64_t xc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    // solo resolutions: same answer as the speculative c* by cause (uncertified / m2 / V), with a
    // remainder, same answer with a remainder, remainder queries valid up to the next failure, whole remainder valid
    uint64_t xc2[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tlast = stamp();
    acc[9] = tlast - t_kernel0;  // pass setup: tree build, registers, first queries
#endif
    // batches awaiting commit, in order: buffer, first query of the buffer,
    // first uncommitted slot, count, iteration of their distance snapshot
    // (two named slots, not arrays: a runtime-indexed array would live in scratch)
    int vq_buf0 = 0, vq_s0 = 0, vq_off0 = 0, vq_n0 = 0, vq_a10 = 0;
    int vq_buf1 = 0, vq_s1 = 0, vq_off1 = 0, vq_n1 = 0, vq_a11 = 0;
    int nvq = 0;
    int cur_buf = 0, cur_s = 0, cur_n = n0;  // batch whose distances are computed this iteration
    // every leaf's exact distance to q (ANN's sequential sum) into sh.dist, from
    // the registers as they are (+inf for slots without a live centroid)
    auto exact_dists = [&](const float* __restrict__ qe) {
        float dv[SL];
#pragma unroll
        for (int s = 0; s < SL; ++s) dv[s] = 0.0f;
#pragma unroll
        for (int d = 0; d < C::DR; ++d) {
            const float qd = qe[d];
#pragma unroll
            for (int s = 0; s < SL; ++s) {
                const float t = fsub(qd, creg[s][d]);
                dv[s] = fadd(dv[s], fmul(t, t));
            }
        }
        if constexpr (C::SPLIT) {  // every leaf's full distance: the tail rows (rare path)
#pragma unroll
            for (int s = 0; s < SL; ++s) {
                const float* tr = trow + (int64_t)(p0 + s) * C::TL;
                if (!((dmask >> s) & 1u))
                    for (int d = 0; d < C::TL; ++d) {
                        const float t = fsub(qe[C::DR + d], tr[d]);
                        dv[s] = fadd(dv[s], fmul(t, t));
                    }
            }
        }
#pragma unroll
        for (int s = 0; s < SL; ++s)
            if (p0 + s < K) sh.dist[p0 + s] = ((dmask >> s) & 1u) ? __builtin_inff() : dv[s];
    };
    int next_load = n0;
    for (int it = 0;; ++it) {
        int ln = opaque_v(lane);  // see opaque_v: refreshed per phase below
#ifdef GSC_STAMPS
        const uint64_t t_it0 = stamp();
        const bool it_bubble = cur_n == 0;  // no new batch: the remainder of a failed one is re-checked
        bool it_fix = false;
#endif
        const bool has_p = nvq > 0;
        const int P_buf = vq_buf0, P_s = vq_s0, P_off = vq_off0, P_n = has_p ? vq_n0 : 0;
        // ---- part 1: chain the pending batch's updates (wave 0); A1(current)
        VPState vst;
#ifdef GSC_STAMPS_PREP
        STAMP(14)  // diagnostic split of "prep": loop top (into a2box's slot) vs the update chain
#endif
        if (wave == 0 && has_p) vp_begin<C>(sh, P_buf, P_off, P_n, vq_a10, ln, lg_pos, lg_tag, vst);
        // The update chain right after its prep, so the V check can start
        // as soon as a wave is done with A1 (wave 0 reaches the mid-A1 barrier
        // early).  C5 -cs4 scan -3.2 % (5551 vs 5732 ms at 128 s) and no VGPR
        // spill left; at D = 16 +0.6 % in round 4 (3361 vs 3342 ms), -1.5 % with
        // round 6's in-batch DFS answers (3221 / 3225 vs 3269 / 3277 ms); D = 32
        // (C3) -2.9 % (2750 / 2768 vs 2836 / 2841 ms)
        constexpr bool kVpEarly = D <= GSC_VP_EARLY_D;
        if constexpr (kVpEarly) {
            if (wave == 0 && has_p) {
                vp_end<C>(sh, P_buf, P_off, P_n, ln, lg_pos, vst, half, it & 1);
                wave_lds_sync();
                if (ln == 0) __hip_atomic_store(&sh.vp_ready, it + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        // prefetch the next batch's queries (they land in LDS in part 3).  Issued
        // after vp_begin: a wait for any later vector-memory op (a scratch reload)
        // waits for this HBM load too, and A1 below issues none
        constexpr int PE = (KB * D + nthreads - 1) / nthreads;
        float pre[PE];
#pragma unroll
        for (int e = 0; e < PE; ++e) {
            const int k = tid + e * nthreads;
            pre[e] = (k < KB * D && next_load + k / D < N) ? X[(int64_t)next_load * D + k] : 0.0f;
        }
        STAMP(0)
        // A1 of the queries in mask m, two per trip: one query's min-tree (a
        // dependent DPP chain) overlaps the other's distance FMAs
        auto a1_mask = [&](uint64_t m) {
#pragma unroll 1
            while (m) {
                const int j0 = __ffsll((long long)m) - 1;
                m &= m - 1;
                const int j1 = m ? __ffsll((long long)m) - 1 : j0;
                if (m) m &= m - 1;
                float dv0[SL], dv1[SL];
                if (C::SPLIT || half)
                    a1_dist_x2<C::H, C::DR, SL>(creg, cn, sh.qm[cur_buf][j0], sh.qm[cur_buf][j1], dv0, dv1);
                else if constexpr (!C::SPLIT)
                    a1_dist_x2<D, D, SL>(creg, cn, sh.qm[cur_buf][j0], sh.qm[cur_buf][j1], dv0, dv1);
                a1_reduce2<C>(dv0, dv1, sh.wrec[vwave][j0], sh.wrec[vwave][j1], vwave, ln);
            }
        };
        const uint64_t curm = cur_n > 0 ? (cur_n >= 64 ? ~0ull : (1ull << cur_n) - 1ull) : 0ull;
#ifdef GSC_STAMPS
        const int cur_n_it = cur_n;
#endif
        uint64_t prunedm = 0;  // queries this wave skipped (wave-uniform)
        float lbp = 0.0f, qn_j = 0.0f, eps_j = 0.0f;  // ln j: query j's box bound, |q|^2, eps
        if constexpr (PRUNE) {
            if (no_prune) {
                a1_mask(curm);
            } else if (cur_n > 0) {
                const int jr = ln < cur_n ? ln : 0;
                const float* qv = sh.q[cur_buf][jr];
                lbp = wave_box_lb<C>(sh, qv, vwave);
                qn_j = half ? norm2_x<C::H>(qv) : norm2_x<D>(qv);
                float M = 0.0f;
#pragma unroll
                for (int w = 0; w < C::NWV; ++w) M = fmaxf(M, sh.cnmax[w]);
                eps_j = fadd(fadd(fmul(fadd(qn_j, M), C::EPSF), 1e-37f), te);
                qn_j = fadd(qn_j, twh);  // |q_h|^2 + TW/2 in half-dimension passes
                // home queries (q inside this wave's box) first: their minima bound
                // the others (a query outside every box is evaluated by all waves)
                const uint64_t home = __ballot(lbp == 0.0f) & curm;
                a1_mask(home);
                wave_lds_sync();
                if ((home >> ln) & 1ull) {
                    const float m = __uint_as_float(sh.wrec[vwave][ln].minbits);
                    const float ubd = fmul(fadd(fadd(qn_j, m), eps_j), 1.0f + 0x1p-20f);
                    atomicMin(&sh.ub[ln], __float_as_uint(fmaxf(ubd, 0.0f)));
                }
#ifdef GSC_STAMPS
                const uint64_t tm0_ = stamp();
                acn[6] += tm0_ - tlast;  // box bounds + home queries
#endif
                lds_barrier();
#ifdef GSC_STAMPS
                {
                    const uint64_t tm1_ = stamp();
                    acn[7] += tm1_ - tm0_;  // the mid-A1 barrier
                    tlast = tm1_;
                }
#endif
                const float ubj = __uint_as_float(sh.ub[jr]);
                const float thr = fmul(fadd(ubj, fmul(4.0f, eps_j)), 1.0f + 0x1p-20f);
                prunedm = __ballot(lbp > thr) & curm & ~home;
#ifdef GSC_STAMPS
                acn[0] += __popcll(home);
                acn[1] += __popcll(prunedm);
                acn[2] += __popcll(curm & ~home & ~prunedm);
#endif
                if ((prunedm >> ln) & 1ull)  // a lower bound of this wave's A1 values (see above)
                    sh.wrec[vwave][ln].minbits = __float_as_uint(fsub(fsub(lbp, fmul(3.0f, eps_j)), qn_j));
                a1_mask(curm & ~home & ~prunedm);
            }
        } else {
            a1_mask(curm);
        }
        if constexpr (!kVpEarly) {
            if (wave == 0 && has_p) vp_end<C>(sh, P_buf, P_off, P_n, ln, lg_pos, vst, half, it & 1);
        }
        {
            STAMP(7)  // slot 7 = the rest of A1 (+ vp_end); slot 1 = the V check below
            if (has_p) {  // V check of the pending batch by the waves done with A1 (v_check_grab)
                if (wave == 0) {
                    if constexpr (!kVpEarly) {
                        wave_lds_sync();
                        if (ln == 0)
                            __hip_atomic_store(&sh.vp_ready, it + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                } else {
                    while (__hip_atomic_load(&sh.vp_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != it + 1)
                        __builtin_amdgcn_s_sleep(1);
                }
                v_check_grab<C>(sh, P_buf, P_off, P_n, ln, it & 1);
            }
        }
#ifdef GSC_STAMPS
        acn[3] += 1;
        acn[5] += P_n;
#endif
        STAMP(1)
        lds_barrier();
        STAMP(6)
        // ---- part 2: commit decision (every wave: the V check is complete) and
        // the next batch's queries, then the certificates of the current batch
        // on the snapshot.  The registers must not change before the fixups:
        // their exact records keep the pruning lower bounds of the waves that
        // skipped a query, which hold for the snapshot only (with post-commit
        // registers a pruned wave's bound could undercut every exact minimum
        // and win the certificate with a record it never wrote).  So the fold
        // follows the fixups, and the log bookkeeping and the residual run
        // after them (part 3), all without the barrier the commit needed before
        // (the fold reads the update chain's rows, not the log).
        ln = opaque_v(ln);
        int fj = -1;
        if (has_p) {
            const uint64_t bad = __ballot(ln < P_n && sh.inval[ln] != 0);
            fj = bad ? __ffsll((long long)bad) - 1 : -1;
        }
        const int kc = has_p ? (fj >= 0 ? fj : P_n) : 0;  // committed prefix of the pending batch
        if (kInBatchDfs && fj >= 0) ib_fail += uniform_int(sh.qrec[P_buf][P_off + fj].valid) == 2 ? 1 : 0;
#ifdef GSC_STAMPS
        int fj_cause = 0;
        if (fj >= 0) {  // why the first failing query failed
            const int cause = sh.inval[fj];
            fj_cause = cause;
            xc2[9] += sh.qrec[P_buf][P_off + fj].valid == 2 ? 1 : 0;  // a DFS answer failed its check
            xc[12] += (cause & 1) ? 1 : 0;
            xc[13] += (cause & 2) ? 1 : 0;
            xc[14] += (cause & 4) ? 1 : 0;
            xc[15] += (cause & 4) && (cause & 3) == 0 ? 1 : 0;
        }
#endif
        if (wave == 0 && fj >= 0 && ln < D) sh.qslow[ln] = sh.q[P_buf][P_off + fj][ln];
        // this iteration's current batch (certificates below); the queue moves on
        const int A_buf = cur_buf, A_n = cur_n;
        // queue bookkeeping (uniform)
        const int solo_j = fj >= 0 ? P_s + P_off + fj : -1;
        if (has_p) {
            if (fj >= 0 && fj + 1 < P_n) {
                vq_off0 = P_off + fj + 1;
                vq_n0 = P_n - fj - 1;
            } else {
                vq_buf0 = vq_buf1;
                vq_s0 = vq_s1;
                vq_off0 = vq_off1;
                vq_n0 = vq_n1;
                vq_a10 = vq_a11;
                --nvq;
            }
        }
        if (cur_n > 0) {
            if (nvq == 0) {
                vq_buf0 = cur_buf;
                vq_s0 = cur_s;
                vq_off0 = 0;
                vq_n0 = cur_n;
                vq_a10 = it;
            } else {
                vq_buf1 = cur_buf;
                vq_s1 = cur_s;
                vq_off1 = 0;
                vq_n1 = cur_n;
                vq_a11 = it;
            }
            ++nvq;
        }
        // next batch of distances: into a free buffer (never the current batch's,
        // whose certificates run below, nor the buffer a failed query's
        // coordinates were copied out of, above)
        cur_n = 0;
        const int freeb = nvq == 0 ? (fj >= 0 ? P_buf ^ 1 : 0) : (nvq == 1 ? vq_buf0 ^ 1 : -1);
        if (freeb >= 0 && !(fj >= 0 && freeb == P_buf) && !(A_n > 0 && freeb == A_buf) && next_load < N) {
            cur_buf = freeb;
            cur_s = next_load;
            cur_n = min(kbe, N - next_load);
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
        if (tid == 0) sh.vc_next = 0;  // the next iteration's V check trips (taken after the A1 barrier)
        if (PRUNE && wave == 0 && ln < KB) sh.ub[ln] = kInfBits;  // the next batch's bounds
        STAMP(4)
        // ---- certificates of the current batch
        if (A_n > 0) {
            // c*'s coordinates, written by the wave that owns c*
            write_cstar<C>(sh, creg, sh.qrec[A_buf], (1ull << A_n) - 1ull, 0, wave, ln, trow);
            STAMP(8)
#pragma unroll 1
            for (int j0 = wave * 4; j0 < A_n; j0 += 4 * NWL)
                a2_group<C, true>(sh, j0, A_n, sh.q[A_buf], sh.qrec[A_buf], 0, nullptr, ln, half, twh, te,
                                  nan_rows != 0
#ifdef GSC_STAMPS
                                  , acc, &tlast, xc
#endif
                );
        }
        // the residual's terms and the cluster ids of the committed prefix, read
        // before the barrier (wave 0 rewrites gp in the next iteration's update chain)
        float err_sq = 0.0f;
        if (wave == kErrWave && ln < kc) err_sq = sqrt_rn(per_col(sh.gp[ln]));
        STAMP(2)
        lds_barrier();
        if (A_n > 0) {
            // queries the approximate certificate could not decide: exact A1 + A2
            // on the snapshot registers (fold_commits runs after the fixups: a
            // pruned wave's lower bound holds for the snapshot only)
            const uint64_t fx = __ballot(ln < A_n && sh.qrec[A_buf][ln].valid == 0);
            if (fx) {
                const int nfx = __popcll(fx);
#ifdef GSC_STAMPS
                it_fix = true;
                acn[4] += nfx;
#endif
                if (wave == 0 && ((fx >> ln) & 1ull)) sh.fxl[__popcll(fx & ((1ull << ln) - 1ull))] = ln;
                uint64_t m = fx;
                while (m) {
                    const int jj = __ffsll((long long)m) - 1;
                    m &= m - 1;
                    if ((prunedm >> jj) & 1ull) {  // still provably far: the exact record's lower bound
                        const float lb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lbp), jj));
                        if (ln == 0) sh.wrec[vwave][jj].minbits = __float_as_uint(lb);
                    } else {
                        a1_query<C>(creg, sh.q[A_buf][jj], sh.wrec[vwave][jj], vwave, ln, dmask, trow, p0,
                                    tw_pass);
                    }
                }
                lds_barrier();
                write_cstar<C>(sh, creg, sh.qrec[A_buf], fx, 0, wave, ln, trow);
#pragma unroll 1
                for (int j0 = wave * 4; j0 < nfx; j0 += 4 * NWL)
                    a2_group<C, false>(sh, j0, nfx, sh.q[A_buf], sh.qrec[A_buf], 0, sh.fxl, ln);
                lds_barrier();
                // Queries the exact certificate cannot decide either: ANN's stale-tree
                // DFS does not provably reach the snapshot's minimum (and mostly does
                // not: 96 % of them resolve elsewhere), or an exact tie.  Their
                // answer on the snapshot is ANN's search itself -- the exact DFS over
                // the snapshot registers (they change only at the fold below) -- and
                // the commit checks it like a certificate: a centroid moved since
                // the snapshot keeps the DFS's improvement sequence when its live
                // distance is not below the best-so-far at its DFS rank
                // (v_check_grab), c* itself when it did not move away (vp_end).
                // Without this such a query fails its commit, is resolved alone and
                // holds the next batch back for an iteration.
                if (kInBatchDfs && 3 * ib_fail <= ib_try + 8) {
                    uint64_t ux = __ballot(((fx >> ln) & 1ull) && sh.qrec[A_buf][ln].valid == 0);
                    const bool any_ux = ux != 0;
                    ib_try += __popcll(ux);
#pragma unroll 1
                    while (ux) {
                        const int jj = __ffsll((long long)ux) - 1;
                        ux &= ux - 1;
                        QRecT<D>& R = sh.qrec[A_buf][jj];
                        exact_dists(sh.q[A_buf][jj]);
                        lds_barrier();  // sh.dist complete
                        int bpos;
                        float key;
                        // NaN passes: NaN and dead leaves are +inf in sh.dist, inert as in the
                        // solo resolution; NaN-first queries are certified (a2_group)
                        if (nan_rows)
                            dfs_parallel_nan<C>(sh, sh.q[A_buf][jj], tid, ln, wave, bpos, key, &R);
                        else
                            dfs_parallel_call<C>(sh, sh.q[A_buf][jj], tid, ln, wave, bpos, key, &R);
                        bpos = uniform_int(bpos);
                        // c*'s snapshot coordinates from its owner; the record from thread 0
                        const int owner_t = bpos >> LS, slot = bpos & (SL - 1);
#pragma unroll
                        for (int s = 0; s < SL; ++s)
                            if (s == slot && tid == owner_t) {
#pragma unroll
                                for (int d = 0; d < C::DR; ++d) R.o[d] = creg[s][d];
                                if constexpr (C::SPLIT)
                                    for (int d = C::DR; d < D; ++d) R.o[d] = trow[(int64_t)bpos * C::TL + (d - C::DR)];
                            }
                        if (tid == 0) {
                            R.cstar = bpos;
                            R.id = sh.t.pidx[bpos];
                            R.g = key;
                            // vp_end's "c* moved: live d < m2" becomes d <= key: a c* that
                            // moved closer stays the DFS's last improvement, and every leaf
                            // after it was at or above key
                            R.m2 = __uint_as_float(__float_as_uint(key) + 1u);
                            R.rate = sh.rate[bpos];
                            R.valid = (R.nimp <= kMaxImp && key <= FLT_MAX) ? 2 : 0;
                        }
#ifdef GSC_STAMPS
                        xc2[8] += 1;
#endif
                    }
                    // the records are complete (the commit's update chain reads R.o next iteration,
                    // at D = 8 before any other barrier)
                    if (any_ux) lds_barrier();
                }
            }
        }
        // every wave folds the committed updates of the centroids it owns, straight
        // from the update chain's rows (no barrier after the commit decision)
        if (kc > 0) fold_commits<C>(sh, creg, cn, cnmax, vwave, ln, P_buf, P_off, kc, it & 1, trow);
#ifdef GSC_BOX_SHRINK
        // experiment: the pruning boxes only grow within a pass (every fold widens
        // them); re-fit them to the registers every GSC_BOX_SHRINK iterations (the
        // next A1's snapshot is these registers; the solo below grows them again)
        if constexpr (!C::SPLIT) {
            if ((it % GSC_BOX_SHRINK) == GSC_BOX_SHRINK - 1) wave_box_init<C>(sh, creg, vwave, ln, p0, dmask);
        }
#endif
        STAMP(3)
        // ---- part 3: bookkeeping of the committed prefix
        ln = opaque_v(ln);
        if (wave == kErrWave && has_p) {
            // cluster ids, counts and the residual in query order (encoder.lpr:743:
            // err += sqrt(best / colCount)) -- beside wave 0's log update
            const int j = ln;
            const bool cj = j < kc;
            const QRecT<D>& R = sh.qrec[P_buf][P_off + (cj ? j : 0)];
            if (cj) {
                clusters[P_s + P_off + j] = R.id;
                atomicAdd(&cnta[R.cstar], 1);
            }
#pragma unroll
            for (int jj = 0; jj < KB; ++jj) {
                const double t = (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(err_sq), jj));
                err = jj < kc ? err + t : err;
            }
        }
        if (wave == 0 && has_p) {
            const int j = ln;
            const bool cj = j < kc;
            const QRecT<D>& R = sh.qrec[P_buf][P_off + (cj ? j : 0)];
            // the last committed update of each centroid becomes its log entry:
            // the entry already holding that centroid, else the r-th free entry
            const bool lastc = cj && sh.nxt[it & 1][j] >= kc && R.pad_ == 0;
            int tgt = lastc ? sh.ient[j] : -1;
            const uint64_t need = __ballot(lastc && tgt < 0);
            const uint64_t freem = __ballot(lg_pos < 0);
            const uint64_t below = (1ull << ln) - 1ull;
            sh.asg[ln] = -1;
            if (lg_pos < 0) sh.freel[__popcll(freem & below)] = ln;
            wave_lds_sync();
            if (lastc && tgt < 0) tgt = sh.freel[__popcll(need & below)];
            if (lastc) {
#pragma unroll
                for (int d = 0; d < D; ++d) sh.lg_c[tgt][d] = sh.newc[it & 1][j][d];
                sh.lg_c[tgt][C::ROW - 1] = sh.newc[it & 1][j][C::ROW - 1];  // |c|^2 (vp_end)
                sh.asg[tgt] = R.cstar;
            }
            wave_lds_sync();
            const int a = sh.asg[ln];
            if (a >= 0) {
                lg_pos = a;
                lg_tag = it;
            }
        }
        if (solo_j >= 0) {
            // the failed query on the live centroids: fresh distances and
            // certificate; exact DFS if the certificate still fails
            ++restarts;
            // a query whose exact certificate already failed on its snapshot
            // (fixup, part 2) goes straight to the exact DFS: the live centroids
            // differ from the snapshot only in the few moved since, and the DFS
            // gives ANN's answer whether or not a new certificate would pass
            // (41 % of the restarts on the C2 frame; the fresh A1 + A2 they skip
            // cost about 10k cycles each)
            const bool snap_failed = uniform_int(sh.qrec[P_buf][P_off + fj].valid) != 1;
            if (!snap_failed) {
                a1_query<C>(creg, sh.qslow, sh.wrec[vwave][KB], vwave, ln, dmask, trow, p0, tw_pass);
                lds_barrier();
                if (wave == 0)
                    a2_group<C, false>(sh, 0, 1, reinterpret_cast<const float(*)[C::QD]>(sh.qslow), &sh.qsolo, KB,
                                       nullptr, ln);
                lds_barrier();
            }
            int bpos;
            float key;
            STAMP(10)
            if (!snap_failed && uniform_int(sh.qsolo.valid)) {
                bpos = uniform_int(sh.qsolo.cstar);
                key = sh.qsolo.g;
            } else {
                exact_dists(sh.qslow);
                // the centroid registers stay live across the DFS (it needs ~40 more
                // VGPRs; parking the 128 in C and reloading them cost 2x the DFS time)
                lds_barrier();  // sh.dist complete
                if (nan_rows) {
                    // NaN leaves carry +inf here: inert, as the query's descent
                    // reaches a real leaf first (NaN-first queries never fail)
                    dfs_parallel_nan<C>(sh, sh.qslow, tid, ln, wave, bpos, key, nullptr);
                } else if constexpr (D <= GSC_DFS_CALL_D) {
                    dfs_parallel_call<C>(sh, sh.qslow, tid, ln, wave, bpos, key, nullptr);
                } else {
                    dfs_parallel<C>(sh, sh.qslow, tid, ln, wave, bpos, key);
                }
                bpos = uniform_int(bpos);
                ++slow_total;
                STAMP(11)
            }
#ifdef GSC_STAMPS
            {
                const bool same = bpos == sh.vcs[fj];
                const bool rem = fj + 1 < P_n;
                const uint64_t badm = __ballot(ln > fj && ln < P_n && sh.inval[ln] != 0);
                const int nb = badm ? __ffsll((long long)badm) - 1 : P_n;
                if (same) {
                    xc2[(fj_cause & 1) ? 0 : ((fj_cause & 2) ? 1 : 2)] += 1;
                    if (rem) {
                        xc2[4] += 1;
                        xc2[5] += (uint64_t)(nb - fj - 1);
                        xc2[6] += nb == P_n ? 1 : 0;
                    }
                }
                xc2[3] += rem ? 1 : 0;
            }
#endif
            // owner publishes c's coordinates; tid 0 moves it (encoder.lpr:735-744);
            // the move enters the log (later batches' snapshots miss it) and the registers
            const int owner_t = bpos >> LS, slot = bpos & (SL - 1);  // owner thread
#pragma unroll
            for (int s = 0; s < SL; ++s)
                if (s == slot && tid == owner_t) {
#pragma unroll
                    for (int d = 0; d < C::DR; ++d) sh.solo_c[d] = creg[s][d];
                    if constexpr (C::SPLIT)
                        for (int d = C::DR; d < D; ++d) sh.solo_c[d] = trow[(int64_t)bpos * C::TL + (d - C::DR)];
                }
            lds_barrier();
            if (wave == kErrWave && ln == 0) err += (double)sqrt_rn(per_col(key));
            if (wave == 0) {
                if (ln == 0) {
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
                if (ln == e) {
                    lg_pos = bpos;
                    lg_tag = it;
#pragma unroll
                    for (int d = 0; d < D; ++d) sh.lg_c[e][d] = sh.solo_c[d];
                    sh.lg_c[e][C::ROW - 1] = half ? norm2_x<C::H>(sh.solo_c) : norm2_x<D>(sh.solo_c);
                }
                sh.pub_pos[ln] = ln == e ? bpos : -1;
            }
            lds_barrier();
            refresh<C>(sh, creg, cn, cnmax, vwave, ln, trow);
        }
        STAMP(5)
#ifdef GSC_STAMPS
        {
            const uint64_t dt_ = stamp() - t_it0;
            xc[it_bubble ? 0 : 2] += 1;
            xc[it_bubble ? 1 : 3] += dt_;
            if (it_fix) {
                xc[4] += 1;
                xc[5] += dt_;
            }
            if (solo_j >= 0) {
                xc[6] += 1;
                xc[7] += dt_;
            }
            xc[8] += (uint64_t)cur_n_it;
        }
#endif
        if (nvq == 0 && cur_n == 0) {
            if (tid == 0) frp->loop_iters = it + 1;
            break;
        }
        if (it > 4 * N + 64) {  // progress guard: every iteration commits or computes
            if (tid == 0) frp->loop_iters = -1;
            guard = true;
            break;
        }
    }
    if (wave == kErrWave && lane == 0) sh.err_out = err;
    __syncthreads();
    err = sh.err_out;
    // write back the live centroids and this pass's counts (cnts[Odd(iter)])
#pragma unroll
    for (int s = 0; s < SL; ++s) {
        const int p = p0 + s;
        if (!((dmask >> s) & 1u)) {
            const int id = sh.t.pidx[p];
#pragma unroll
            for (int d = 0; d < C::DR; ++d) C_[(int64_t)id * D + d] = creg[s][d];
            if constexpr (C::SPLIT)
                for (int d = C::DR; d < D; ++d) C_[(int64_t)id * D + d] = trow[(int64_t)p * C::TL + (d - C::DR)];
        }
    }
    for (int p = tid; p < K; p += nthreads) {  // the commits' atomics live in L2: read past this CU's L1
        const int id = sh.t.pidx[p];
        if (id != 0xFFFF) prev_cnt[id] = __hip_atomic_load(&cnta[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#ifdef GSC_STAMPS
    if (lane == 0)
        for (int k = 0; k < 16; ++k) frp->stamps[wave * 16 + k] += acc[k];
    if (lane == 0)
        for (int k = 0; k < 8; ++k) frp->acounts[wave * 8 + k] += acn[k];
    if (tid == 0)
        for (int k = 0; k < 16; ++k) frp->xcounts[k] += xc[k];
    if (tid == 0)
        for (int k = 0; k < 16; ++k) frp->xcounts2[k] += xc2[k];
#endif
    const double diff = err > prev_err ? err - prev_err : prev_err - err;
    const bool done = diff <= tol || pass + 1 >= kMaxScanIters || guard;
    prev_err = err;
    if (tid == 0) {
        frp->iters = pass + 1;
        frp->slow += slow_total;
        frp->restarts += restarts;
        frp->err = err;
        frp->done = done ? 1 : 0;
        if (done) frp->t_done = __builtin_amdgcn_s_memrealtime();  // diagnostic: the scan tail
    }
    // the next pass's tree build and rate lookups read C and prev_cnt as
    // written above by other lanes
    __threadfence();
    __syncthreads();
    if (done) {
        // hand the final clusters to the host's post-processing while the
        // other frames still scan: a host-mapped copy, then the flag
        int* clh = uniform_ptr(frp->cl_host);
        if (clh) {
            for (int j = tid; j < N; j += nthreads)
                clh[j] = __hip_atomic_load(&clusters[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __threadfence_system();
            __syncthreads();
            if (tid == 0) __hip_atomic_store(uniform_ptr(frp->notify), 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        break;
    }
    }
    }
}

}  // namespace gsc

using namespace gsc;

template <class C>
static hipError_t launch_scan(ReduceFrame* frames, int nframes, const float* X, float* Cc, int* is,
                              const float* rate_tab, double tol, int max_passes, int opts, float* tails,
                              hipStream_t st) {
    const size_t shm = sizeof(Scan2Shared<C>);
    static_assert(sizeof(Scan2Shared<C>) <= 160 * 1024, "LDS budget (160 KB per CU)");
    hipError_t e = hipFuncSetAttribute((const void*)scan_batch_kernel<C>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)shm);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(scan_batch_kernel<C>, dim3(nframes), dim3(C::NT), shm, st, frames, nframes, X, Cc, is, rate_tab,
                       tol, max_passes, opts, tails);
    return hipGetLastError();
}

// Batched KNNScanReduce for every frame (K <= 2^logk, 2^logk in 256..4096; a
// frame's own K (frp->K) below 2^logk runs the padded layout; D = 8, 16 or 32,
// D = 32 with K = 4096 in the split layout): each frame runs its passes from
// frp->iters until it converges, reaches max_passes or meets a NaN pass (left
// to the generic kernel).  Returns hipErrorInvalidValue for shapes it does not
// cover.
extern "C" hipError_t gsc_launch_scan_batch(int D, int logk, ReduceFrame* frames, int nframes, const float* X,
                                            float* Cc, int* is, const float* rate_tab, double tol, int max_passes,
                                            int opts, float* tails, hipStream_t st) {
#define SB(DV, LK, SLV)                                                                                           \
    if (D == DV && logk == LK)                                                                                    \
        return launch_scan<ScanCfg<DV, LK, SLV>>(frames, nframes, X, Cc, is, rate_tab, tol, max_passes, opts, tails, \
                                                 st);
    // K below 4096: fewer leaves per lane, so a frame keeps (up to) 8 waves --
    // the per-search work there is latency (A2 certificates, V checks and the
    // commit spread over the waves): K = 256 / 512 one leaf per lane (4 / 8
    // waves), K = 1024 two, K = 2048 four
    SB(8, 8, 1) SB(8, 9, 1) SB(8, 10, 2) SB(8, 11, 4) SB(8, 12, 8)
    SB(16, 8, 1) SB(16, 9, 1) SB(16, 10, 2) SB(16, 11, 4) SB(16, 12, 8)
    SB(32, 8, 1) SB(32, 9, 1) SB(32, 10, 2) SB(32, 11, 4)
    // D = 32, K = 4096: the DCT half of every centroid in VGPRs and the
    // cepstrum half in the frame's tail array (split layout; measured at D = 16
    // too: 4294 vs 4309 ms at the C2 bench shape, not kept)
    if (D == 32 && logk == 12)
        return launch_scan<ScanCfg<32, 12, 8, 16>>(frames, nframes, X, Cc, is, rate_tab, tol, max_passes, opts, tails,
                                                   st);
#undef SB
    return hipErrorInvalidValue;
}

extern "C" size_t gsc_scan_tail_floats_per_frame(int D, int logk) {
    return logk == 12 && D == 32 ? 4096 * size_t(D / 2) : 0;
}
