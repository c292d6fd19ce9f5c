// Host side of the MI355X SoundChunks encoder: the TEncoder/TFrame pipeline
// of reference encoder/encoder.lpr around the GPU hot path.
//
//   host  : Load + PrepareFrames (encoder.lpr:1111-1152, 1294-1429),
//           FindAttenuationDivider (566-605), MakeChunks features (349-485),
//           cluster means + FPC QuickSort (843-889), KNNFit pruning/sort
//           (970-977), SaveStream bit packing (980-1107)
//   device: yakmo seeding, KNNScanReduce, KNNFit search (gsc_kernels.hip)
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/soundchunks.h"

namespace gsc {

struct FrameState {
    int index = 0, start = 0, sample_count = 0;
    int atten_div = 6;
    int n = 0;                 // chunkRefs count (chunk-major, channel-minor)
    std::vector<double> src;   // n*CS srcData
    std::vector<float> feat;   // n*2CS Single(dct)
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

class Encoder {
   public:
    explicit Encoder(const gsc_options& o) : opt_(o) {}
    // Load + PrepareFrames; returns 0 or a negative error code
    int prepare(const uint8_t* wav, size_t len, std::string* err);
    int frame_count() const { return int(fr_start_.size()); }
    // Encode frames [b, e) and return their concatenated stream bytes
    int encode_range(int b, int e, std::vector<uint8_t>* out, std::string* err, gsc_timing* tim);

    int channels() const { return channels_; }
    int sample_rate() const { return sample_rate_; }
    long long sample_count() const { return sample_count_; }

   private:
    void frame_host_prepare(FrameState& f) const;
    void frame_reduce_post(FrameState& f, bool reduced) const;
    void frame_knnfit_post(FrameState& f) const;
    void frame_save(FrameState& f) const;

    gsc_options opt_;
    int channels_ = 0, sample_rate_ = 0;
    int sample_count_ = 0;
    int block_ = 1;
    std::vector<std::vector<double>> filtered_;  // [ch][sample] = s / 32767
    std::vector<int> fr_start_, fr_end_;
};

}  // namespace gsc
