// Host side of the MI355X SoundChunks encoder: the TEncoder/TFrame pipeline
// of reference encoder/encoder.lpr around the GPU hot path.
//
//   host  : Load + PrepareFrames (encoder.lpr:1111-1152, 1294-1429),
//           cluster means + FPC QuickSort (843-889), KNNFit pruning/sort by
//           use count (970-977), SaveStream header and codebook (980-1048)
//   device: FindAttenuationDivider (566-605) and the MakeChunks features
//           (349-485, gsc_dsp.hip), yakmo seeding (gsc_yakmo.hip),
//           KNNScanReduce (gsc_scan.hip), KNNFit search (gsc_kernels.hip),
//           use counts and the SaveStream index bitstream (1050-1106,
//           gsc_pack.hip), reconstruction (gsc_recon.hip)
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <utility>
#include <string>
#include <vector>

#include "../../include/soundchunks.h"

namespace gsc {

// allocator whose value-initialisation is a no-op: large host buffers are
// filled (and first touched) by the parallel workers, not by one thread
template <typename T>
struct NoInitAlloc : std::allocator<T> {
    template <typename U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <typename U>
    NoInitAlloc(const NoInitAlloc<U>&) {}
    template <typename U>
    void construct(U* p) noexcept {
        ::new (static_cast<void*>(p)) U;
    }
    template <typename U, typename... A>
    void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};

// host worker pool (gsc_runtime.cpp): fn(0..n-1) on up to `threads` threads
void parallel_for(int n, int threads, const std::function<void(int)>& fn);
int host_threads();

struct FrameState {
    int index = 0, start = 0, sample_count = 0;
    int atten_div = 6;
    int n = 0;                 // chunkRefs count (chunk-major, channel-minor)
    std::vector<uint8_t> neg, rev;
    std::vector<int> red;      // final reduced-chunk index per chunk
    // reduced chunks
    int r = 0;
    int r_before_prune = 0;  // reducedChunks.Count at KNNFit time
    std::vector<double> rsrc;
    std::vector<int16_t> rdst;
    std::vector<uint8_t> ratten, rneg;
    // Reduce outputs (device)
    std::vector<float> cent;   // K*2CS
    std::vector<int> clusters; // N
    int scan_iters = 0, scan_slow = 0;
    // KNNFit
    std::vector<int> best;     // N
    std::vector<uint8_t> stream;
};

// Builds the exact FPC trig tables for chunk size cs (not thread-safe: call
// before starting per-frame workers).
void warm_trig_tables(int cs);
// The same tables packed for the device DSP: dct, dft cos, dft sin, idft cos,
// idft sin (cs*cs f64 each), plus the DCT scale factors sqrt(1/2), sqrt(2/cs).
void trig_pack(int cs, std::vector<double>* tab, double* s0, double* scale);

// Reconstruction request of an encode: the 16-bit signal
// the reference rebuilds after MakeFrames (encoder.lpr:2019-2027), written
// into pcm (interleaved [sample][channel], the padded SampleCount), and the
// exact integer sum of (srcData - dstData)^2 over the encoded frames (the
// numerator of ComputePsyADelta, encoder.lpr:1862-1880).
struct ReconOut {
    int16_t* pcm = nullptr;
    const uint8_t* wav = nullptr;  // the source WAV (srcData for PsyADelta)
    size_t wav_len = 0;
    unsigned long long sq = 0;
    double ms = 0;
};

// device slabs + stream of the KNNFit/packing pipeline of one encode (gsc_runtime.cpp)
struct PostCtx;

// -py reducer (gsc_birch_host.cpp): cluster.py's Birch labels of N samples
int birch_reduce_labels(int n, int d, const float* feat, int K, int* labels, std::string* err);

class Encoder {
   public:
    explicit Encoder(const gsc_options& o) : opt_(o) {}
    // Load + PrepareFrames; returns 0 or a negative error code
    int prepare(const uint8_t* wav, size_t len, std::string* err);
    // frame boundaries computed elsewhere (starts/ends of all nframes frames);
    // only the samples of frames [b, e) are loaded
    int prepare_bounds(const uint8_t* wav, size_t len, const int* starts, const int* ends, int nframes, int b, int e,
                       std::string* err);
    const std::vector<int>& frame_starts() const { return fr_start_; }
    const std::vector<int>& frame_ends() const { return fr_end_; }
    // a batch of WAVs (same channel count, sample rate and ChunksPerFrame) as
    // one frame list: each file's own Load + PrepareFrames, the files' padded
    // samples back to back, frames of file f from file_first()[f]
    int prepare_many(const uint8_t* const* wavs, const size_t* lens, int nfiles, std::string* err);
    const std::vector<int>& file_first() const { return file_first_; }
    int frame_count() const { return int(fr_start_.size()); }
    // chunkRefs count of frame i: chunks x channels (encoder.lpr:467-485)
    int frame_chunks(int i) const {
        const int sc = fr_end_[size_t(i)] - fr_start_[size_t(i)] + 1;
        return ((sc - 1) / opt_.chunk_size + 1) * channels_;
    }
    // Encode frames [b, e) and return their concatenated stream bytes
    int encode_range(int b, int e, std::vector<uint8_t>* out, std::string* err, gsc_timing* tim,
                     ReconOut* recon = nullptr, std::vector<size_t>* frame_bytes = nullptr);
    // Device DSP of frame f alone (parity tests): attenuation divider and the
    // N x 2CS features
    int dsp_frame(int f, int* atten_div, std::vector<float>* feat, std::string* err);

    int channels() const { return channels_; }
    int sample_rate() const { return sample_rate_; }
    long long sample_count() const { return sample_count_; }

   private:
    // Load: header, geometry, the samples of [s0, s1) into pcm_
    int load(const uint8_t* wav, size_t len, int64_t s0, int64_t s1, std::string* err);
    // PrepareFrames pass 2: power sums and the frame cut (needs the whole file loaded)
    int plan(std::string* err);
    void cut_frames(const double* pw, double per_frame);
    void frame_host_src(FrameState& f) const;  // chunk count (encoder.lpr:467-485)
    void chunk_src(const FrameState& f, int j, double* out) const;  // chunk j's srcData (CS doubles)
    // device DSP for frames (first frame index b): atten_div, neg / rev on the
    // host side, features left in the device slab *dX at (*xoff)[i]; with dQ,
    // also the KNNFit queries Single(srcData) (N*CS floats per frame, frames
    // concatenated) in the device slab *dQ
    int device_dsp(int b, std::vector<FrameState>& frames, void* dX, std::vector<int64_t>* xoff, double* ms,
                   std::string* err, void* dQ = nullptr);
    // reconstruction of frames [b, b + frames.size()) on the device (after KNNFit)
    int device_recon(int b, const std::vector<FrameState>& frames, ReconOut* ro, std::string* err);
    void frame_reduce_post(FrameState& f, bool reduced) const;
    // KNNFit prune + sort by use count (use[r] in, remap[r] out)
    void frame_prune(FrameState& f, const int* use, int* remap) const;
    // SaveStream's header, attenuations and dstData (the index stream is packed on the device)
    void frame_save_head(FrameState& f) const;
    // KNNFit, prune/sort and index packing of frames ids (gsc_runtime.cpp)
    int post_group(std::vector<FrameState>& frames, const std::vector<int>& ids, const std::vector<char>& reduced,
                   PostCtx& ctx, std::string* err);

    gsc_options opt_;
    int channels_ = 0, sample_rate_ = 0;
    int sample_count_ = 0;   // SampleCount, padded to whole blocks
    int file_samples_ = 0;   // sample frames in the WAV
    int frame_count_est_ = 0;  // FrameCount before the cut (encoder.lpr:1335)
    int block_ = 1;
    int64_t pcm_off_ = 0;    // first sample held in pcm_
    std::vector<int16_t, NoInitAlloc<int16_t>> pcm_;  // [sample - pcm_off_][ch] SmallInt, zero padded (srcData * 32767)
    std::vector<int> fr_start_, fr_end_;
    std::vector<int> file_first_{0};  // first frame of each file (+ the total), one file unless prepare_many
};

}  // namespace gsc
