// SoundChunks MI355X encode hot path -- device-side descriptors shared by the
// HIP kernels (gsc_kernels.hip) and the host runtime (gsc_runtime.cpp).
//
// All arrays live in HBM, one slab per batch of frames; a descriptor per frame
// holds offsets into those slabs (no per-frame allocations).
#pragma once
#include <stdint.h>

namespace gsc {

constexpr int kMaxK = 4096;        // CMaxChunksPerFrame (encoder.lpr:15)
constexpr int kMaxInternal = 4095; // internal kd nodes for K <= 4096 (heap index < 4095)
constexpr int kScanThreads = 512;  // 8 waves, 2 per SIMD
constexpr int kScanSlots = 8;      // kd leaves (centroids) per lane, 512*8 = 4096
constexpr int kMaxScanIters = 100; // CMaxIterations (encoder.lpr:703)
constexpr int kMaxChunkSize = 16;  // ChunkSize up to 16: 2*CS <= 32 features (-cs is unclamped, encoder.lpr:1992)

// Row stride of the feature slab (Dataset, encoder.lpr:799-806) for a
// ChunkSize: the 2*CS features padded with zeros to the next kernel width
// 8 / 16 / 32.  Trailing zero features change no f32 distance, norm, mean or
// move (x + 0*0 = x, (0 - 0)*rate + 0 = 0, exactly), ANN never splits on a
// zero-spread dimension while a real one has spread (annMaxSpread keeps the
// first maximum), and the residual divides by the real colCount (dcol), so
// the padded search is the reference's search on the real features.
__host__ __device__ constexpr int feature_stride(int cs) { return 2 * cs <= 8 ? 8 : (2 * cs <= 16 ? 16 : 32); }

// IEEE (correctly rounded) f32 sqrt, as the reference's SSE sqrtss.  HIP's
// __fsqrt_rn is __ocml_native_sqrt_f32 -- a bare v_sqrt_f32, 1 ulp -- unless
// OCML_BASIC_ROUNDED_OPERATIONS is defined; __builtin_sqrtf lowers to
// v_sqrt_f32 plus the +-1 ulp fma correction.  One ulp flips KNNFit's
// SameValue-within-eps ties (encoder.lpr:955-962) and ScanReduce's err sum.
__device__ inline float sqrt_rn(float x) { return __builtin_sqrtf(x); }

// One frame of TFrame.Reduce / KNNScanReduce work (encoder.lpr:785-913, 699-765).
struct ReduceFrame {
    int64_t x_off;        // Dataset: N*D floats at X + x_off (row major)
    int64_t c_off;        // Centroids: K*D floats at C + c_off (yakmo out, scan in/out)
    int64_t n_off;        // per-point scratch (N): clusters, d0, id, cum at +n_off
    int64_t k_off;        // per-centroid scratch (K): previous-pass counts by centroid id
    int64_t ka_off;       // per-centroid scratch (K): this pass's counts by kd-leaf position
    int64_t t_off;        // split layout (D = 32, K = 4096): the tail features, K x 16 floats at T + t_off
    int32_t N, K;
    int32_t iters;        // out: KNNScanReduce passes
    int32_t slow;         // out: searches resolved by the exact DFS fallback
    double err;           // residual of the last pass (encoder.lpr:743)
    int32_t done;         // SameValue(err, prevErr, 10^-Precision) or 100 passes
    int32_t generic;      // this pass needs the generic kernel (NaN centroids)
    int32_t restarts;     // out: batched-pipeline restarts (diagnostic)
    int32_t loop_iters;   // out: batched-pipeline iterations (diagnostic); -1 = guard tripped
    int32_t tree_exact;   // out: passes whose kd-tree needed the sequential build (median ties)
    int32_t dcol;         // colCount = 2*ChunkSize (the residual's divisor, encoder.lpr:743); 0 = the slab width
    uint64_t t_done;      // out: s_memrealtime (100 MHz) when the batched kernel finished the frame
    // optional (batched kernel): when the frame is done, its final clusters are
    // copied to cl_host (host-mapped, N ints) and then *notify is set (system
    // scope), so the host post-processes it while other frames still scan
    int32_t* cl_host;
    int32_t* notify;
    uint64_t stamps[128]; // out (GSC_STAMPS builds only): per-phase cycles, 16 per wave
    uint64_t ystamps[16]; // out (GSC_STAMPS builds only): yakmo phase cycles (gsc_yakmo.hip)
    uint64_t acounts[64]; // out (GSC_STAMPS builds only): per wave, A1 queries home / pruned / evaluated, iterations, fixups, pending size
    uint64_t xcounts[16]; // out (GSC_STAMPS builds only, wave 0): iteration kinds and their cycles (gsc_scan.hip)
    uint64_t xcounts2[16]; // out (GSC_STAMPS builds only, wave 0): solo resolutions against the speculative answer
};

// One frame of the encoder's per-frame DSP: FindAttenuationDivider
// (encoder.lpr:566-605) and the MakeChunks features (encoder.lpr:467-485).
struct DspFrame {
    int64_t s_off;        // first sample of the frame in each channel row of the sample slab
    int64_t x_off;        // features out: n*feature_stride(CS) floats at X + x_off (chunk-major, channel-minor)
    int64_t c_off;        // per-chunk bytes out (neg | rev << 1) at +c_off
    int32_t sc;           // frame sample count
    int32_t n;            // chunks (chunk_count * channels)
    int32_t atten_div;    // out: FindAttenuationDivider
    int32_t pad_;
};

// One frame of the reconstruction (TBand.MakeDstData, encoder.lpr:487-522).
struct ReconFrame {
    int64_t chunk_off;    // n chunk words (final reduced index << 2 | neg << 1 | rev) at +chunk_off
    int64_t red_off;      // final reduced chunks: r*CS int16 at rdst + red_off*CS, attenuation at +red_off
    int64_t out_off;      // the frame's first sample, relative to the batch's first sample
    int32_t n, sc;        // chunkRefs count, frame sample count
    double law;           // AttenuationLaw = 1 / AttenuationDivider
};

// One frame of TFrame.KNNFit (encoder.lpr:915-978).
struct FitFrame {
    int64_t cand_off;     // R*CS floats: forward candidate values (neg/rev derived)
    int64_t q_off;        // N*CS floats: queries Single(srcData)
    int64_t out_off;      // N ints: best candidate index f = 4c + 2neg + rev
    int32_t R, N;
    float eps;
    int32_t overflow;     // out: queries whose tie set exceeds ANN's 64-NN bucket
};

// One frame of the KNNFit post-processing and SaveStream's index bitstream
// (gsc_pack.hip; encoder.lpr:966-977, 1044-1106).
struct PackFrame {
    int64_t out_off;      // N ints: KNNFit best (4c + 2neg + rev) at best + out_off
    int64_t r_off;        // R ints: use counts (out) / old -> new index map (in) at + r_off
    int64_t w_off;        // bitstream: pack_word_capacity(N) zeroed u32 words at words + w_off
    int32_t N, R;         // chunkRefs count, reducedChunks count before pruning (-pr0 passthrough: N)
    int32_t nbits;        // out: bits of the stream (16-bit words written = ceil(nbits / 16))
    int32_t pad_;
};

// u32 words that hold the index stream of n chunks (<= 17 bits per code)
inline int64_t pack_word_capacity(int64_t n) { return (n * 17 + 31) / 32 + 1; }

// ANN kd-tree (ANN_KD_STD, bs = 1) over n points, heap-indexed split nodes
// (gsc_ann.hip): the drop-in ABI's trees and the KNNFit candidate trees.
struct AnnTree {
    const float* pts;  // n * dd, row major (the live point values)
    int n, dd;
    int* pidx;         // n
    int* cd;           // heap-indexed split data, 2 * pow2ceil(n) entries
    float* cv;
    float* lo;
    float* hi;
    float* bnd;        // 2 * dd: bounding rect lo | hi
    float* val;        // n floats of build scratch (the staged cut values)
    int ncap;          // entries of cd / cv / lo / hi (0: unchecked; the KNNFit overflow replay sets it)
};

// One KNNFit query whose tie set exceeds ANN's 64-NN bucket: replayed through
// ANN's priority search over its frame's candidate tree (gsc_ann.hip).
struct KnnOvJob {
    int tree;   // index into the tree array
    int q_off;  // query: dd floats at q + q_off
    int out;    // result slot
    float eps;  // SameValue epsilon of the frame (encoder.lpr:940-943)
};

}  // namespace gsc
