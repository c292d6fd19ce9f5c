// Host stages of the encoder (see gsc_encoder.h).  Each function cites the
// reference encoder/encoder.lpr lines it reproduces bit-exactly.
#include "gsc_encoder.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "fpc_math.h"
#include "gsc_device.h"
#include "gsc_seqsum.h"

namespace gsc {
namespace {

constexpr int kMaxAttenuation = 15;  // CMaxAttenuation (encoder.lpr:14)

// coeff(a) = 1 + sum_{i=0..a} i*law, accumulated left to right (encoder.lpr:1654-1656)
inline double atten_coeff(int a, double law) {
    double c = 1.0;
    for (int i = 0; i <= a; ++i) c += double(i) * law;
    return c;
}

// TEncoder.makeOutputSample (encoder.lpr:1648-1663)
inline int16_t output_sample(double smp, int obd, double coeff, bool neg) {
    int16_t s16 = int16_t(fpc::round(smp * double(obd) * coeff));
    if (neg) s16 = int16_t(-int(s16));
    int v = s16;
    v = std::max(v, -obd + 1);
    v = std::min(v, obd - 1);
    return int16_t(v);
}

// TEncoder.makeFloatSample (encoder.lpr:1665-1680)
inline double float_sample(int16_t smp, double obd, double coeff, bool neg) {
    int16_t s16 = smp;
    if (neg) s16 = int16_t(-int(s16));
    double r = double(s16) / (obd * coeff);
    if (r < -1.0) r = -1.0;
    if (r > 1.0) r = 1.0;
    return r;
}

// hiSmp of TEncoder.ComputeAttenuation (encoder.lpr:1687-1689)
inline int64_t hi_sample(const double* s, int cs) {
    int64_t hi = 0;
    for (int i = 0; i < cs; ++i) hi = std::max(hi, fpc::ceil_pos(std::fabs(s[i] * 32767.0)));
    return hi;
}

// ComputeAttenuation loop (encoder.lpr:1691-1697) given hiSmp
inline int attenuation_of(int64_t hi, double law) {
    int r = 0;
    double coeff = 1.0;
    do {
        ++r;
        coeff += double(r) * law;
    } while (!((double(hi) * coeff > 32767.0) || (r > kMaxAttenuation)));
    return r - 1;
}

// TChunk.ComputeDstAttributes sign/reverse heuristics (encoder.lpr:374-396)
inline void sign_reverse(const double* s, int cs, bool* neg, bool* rev) {
    double p1 = 0.0, p2 = 0.0;
    for (int i = 0; i < cs; ++i)
        if (s[i] < 0) p1 -= s[i];
    for (int i = 0; i < cs; ++i)
        if (s[i] > 0) p2 += s[i];
    *neg = p1 > p2;
    p1 = 0.0;
    p2 = 0.0;
    for (int i = 0; i < cs / 2; ++i) p1 += std::fabs(s[i]);
    for (int i = cs / 2; i < cs; ++i) p2 += std::fabs(s[i]);
    *rev = p1 > p2;
}

// exact FPC trig values for every angle the features use
struct TrigTables {
    int cs = 0;
    std::vector<double> dct, dft_c, dft_s, idft_c, idft_s;
};

const TrigTables& trig_for(int cs) {
    static TrigTables cache[17];
    static bool ready[17] = {false};
    TrigTables& t = cache[cs];
    if (!ready[cs]) {  // built before worker threads start (Encoder::encode_range)
        const double PI = 3.14159265358979323846;
        t.cs = cs;
        t.dct.resize(size_t(cs) * cs);
        t.dft_c.resize(size_t(cs) * cs);
        t.dft_s.resize(size_t(cs) * cs);
        t.idft_c.resize(size_t(cs) * cs);
        t.idft_s.resize(size_t(cs) * cs);
        for (int k = 0; k < cs; ++k)
            for (int n = 0; n < cs; ++n) {
                t.dct[k * cs + n] = fpc::cos(PI / double(cs) * (double(n) + 0.5) * double(k));
                const double a = ((-2.0 * PI) * double(k)) * double(n) / double(cs);
                t.dft_c[k * cs + n] = fpc::cos(a);
                t.dft_s[k * cs + n] = fpc::sin(a);
                const double b = ((2.0 * PI) * double(k)) * double(n) / double(cs);
                t.idft_c[k * cs + n] = fpc::cos(b);
                t.idft_s[k * cs + n] = fpc::sin(b);
            }
        ready[cs] = true;
    }
    return t;
}

// FPC TFPSList.QuickSort (encoder.exe @0x10003d410) on `items`, count descending
void fpc_quicksort(int* items, const int* count, int L, int R) {
    int I, J, P;
    do {
        I = L;
        J = R;
        P = (L + R) >> 1;
        do {
            const int pivot = count[items[P]];
            while (count[items[I]] > pivot) ++I;
            while (count[items[J]] < pivot) --J;
            if (I <= J) {
                std::swap(items[I], items[J]);
                if (P == I) P = J;
                else if (P == J) P = I;
                ++I;
                --J;
            }
        } while (I <= J);
        if (L < J) fpc_quicksort(items, count, L, J);
        L = I;
    } while (I < R);
}

}  // namespace

void warm_trig_tables(int cs) { (void)trig_for(cs); }

void trig_pack(int cs, std::vector<double>* tab, double* s0, double* scale) {
    const TrigTables& t = trig_for(cs);
    tab->clear();
    for (const auto* v : {&t.dct, &t.dft_c, &t.dft_s, &t.idft_c, &t.idft_s}) tab->insert(tab->end(), v->begin(), v->end());
    *s0 = std::sqrt(0.5);
    *scale = std::sqrt(2.0 / double(cs));
}

// TEncoder.Load (encoder.lpr:1111-1152) and the option / geometry part of
// PrepareFrames (encoder.lpr:1241-1351): header, SampleCount padded to whole
// blocks, the -br ChunksPerFrame search.  The SmallInt samples of [s0, s1)
// (zero past the file's end) are copied into pcm_.
int Encoder::load(const uint8_t* wav, size_t len, int64_t s0, int64_t s1, std::string* err) {
    if (len < 44) {
        *err = "WAV shorter than its 44-byte header";
        return -1;
    }
    sample_rate_ = int(uint32_t(wav[0x18]) | (uint32_t(wav[0x19]) << 8) | (uint32_t(wav[0x1a]) << 16) |
                       (uint32_t(wav[0x1b]) << 24));
    channels_ = int(wav[0x16] | (wav[0x17] << 8));
    if (channels_ <= 0 || sample_rate_ <= 0) {
        *err = "invalid channel count or sample rate";
        return -1;
    }
    const gsc_options& o = opt_;
    if (o.chunk_blend != 0) {
        *err = "ChunkBlend != 0 is not supported (decoder.lpr asserts it is 0)";
        return -2;
    }
    if (!(o.chunk_bit_depth == 8 || o.chunk_bit_depth == 12)) {
        *err = "ChunkBitDepth must be 8 or 12 (TFrame.SaveStream)";
        return -2;
    }
    // -cs is unclamped in the reference (encoder.lpr:1992); the kernels take
    // 2*ChunkSize <= 32 features (padded to 8 / 16 / 32, gsc_device.h feature_stride)
    if (o.chunk_size < 1 || o.chunk_size > kMaxChunkSize) {
        *err = "ChunkSize must be 1..16 (2*ChunkSize <= 32 features)";
        return -2;
    }
    const int cs = o.chunk_size, ch = channels_;
    const int64_t sc64 = int64_t((len - 44) / (2 * size_t(ch)));
    if (sc64 > int64_t(INT32_MAX) / 2) {
        *err = "sample count out of range";
        return -1;
    }
    const int sc = int(sc64);
    const double hc = std::min(o.high_cut, double(sample_rate_) / 2);
    const double fcl = o.low_cut / double(sample_rate_), fch = hc / double(sample_rate_);
    if (fcl > 0.0 || fch < 0.5) {
        *err = "band-pass filtering (-lc/-hc below Nyquist) is not supported";
        return -2;
    }
    const int under = int(std::max<int64_t>(1, fpc::round(0.25 / fch)));
    block_ = under * (cs - o.chunk_blend);
    sample_count_ = ((sc - 1) / block_ + 1) * block_;  // Pascal div truncates
    file_samples_ = sc;
    const int SC = sample_count_;
    frame_count_est_ = int(fpc::ceil_pos(double(SC) / (double(sample_rate_) * (o.frame_length / 1000.0))));
    // ChunksPerFrame search only changes anything with -br (encoder.lpr:1337-1351)
    if (o.bit_rate > 0) {
        int cpf = o.chunks_per_frame;
        const long long projected =
            (long long)std::ceil((double(SC) / double(sample_rate_)) * (double(o.bit_rate) * 1024.0 / 8.0));
        ++cpf;
        for (;;) {
            --cpf;
            const double band = (double(SC) * double(ch) * (std::log2(double(cpf)) + 3 + 1 + 1)) /
                                (8.0 * double(cs - o.chunk_blend) * double(under));
            const double frame = double(cpf * cs) * double(o.chunk_bit_depth) / 8.0 + double(cpf) * 4.0 / 8.0 + 16;
            const int32_t tent = int32_t(fpc::round(0.0 + band * 0.8 + double(frame_count_est_) * frame));
            if (tent <= projected || cpf <= 1) break;
        }
        opt_.chunks_per_frame = cpf;
    }
    // the samples of [s0, s1): a straight copy of the little-endian PCM16
    // (zero past the file, PrepareFrames pads SampleCount, encoder.lpr:1317-1323)
    s0 = std::max<int64_t>(0, s0);
    s1 = std::min<int64_t>(SC, s1);
    pcm_off_ = s0;
    const int64_t n = std::max<int64_t>(s1 - s0, 1);
    pcm_.resize(size_t(n) * size_t(ch));
    const int64_t have = std::max<int64_t>(0, std::min<int64_t>(s1, sc) - s0);
    constexpr int64_t kBlk = int64_t(1) << 18;
    const int nblk = int((n + kBlk - 1) / kBlk);
    const uint8_t* d = wav + 44;
    parallel_for(nblk, host_threads(), [&](int k) {
        const int64_t a = int64_t(k) * kBlk, b = std::min(n, a + kBlk);
        const int64_t c = std::min(b, have);
        if (c > a) std::memcpy(pcm_.data() + size_t(a) * ch, d + size_t(s0 + a) * ch * 2, size_t(c - a) * ch * 2);
        if (b > std::max(a, c))
            std::memset(pcm_.data() + size_t(std::max(a, c)) * ch, 0, size_t(b - std::max(a, c)) * ch * 2);
    });
    return 0;
}

// PrepareFrames pass 2 (encoder.lpr:1374-1425): avgPower, totalPower and the
// RMS-power balanced frame cut, every f64 sum bit-identical to the
// reference's sequential loops -- evaluated in parallel (gsc_seqsum.h) and,
// for the cut, by speculating the frame boundaries from an approximate
// prefix and verifying every frame's exact running sum.
int Encoder::plan(std::string* err) {
    const int SC = sample_count_, ch = channels_;
    if (pcm_off_ != 0 || int64_t(pcm_.size()) < int64_t(SC) * ch) {
        *err = "PrepareFrames needs the whole file loaded";
        return -1;
    }
    const int16_t* pcm = pcm_.data();
    const int T = host_threads();
    const bool tm = std::getenv("GSC_HOST_TIMING") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto q0 = now();
    SeqSumStats st_avg, st_tot;
    auto par = [&](int n, const std::function<void(int)>& fn) { parallel_for(n, T, fn); };
    // Sqr(makeFloatSample(srcData)) per SmallInt value, srcData = s / 32767
    static const std::vector<double> sq = [] {
        std::vector<double> t(65536);
        for (int v = -32768; v < 32768; ++v) {
            const double f = double(v) / 32767.0;
            t[size_t(v + 32768)] = f * f;
        }
        return t;
    }();
    const double* SQ = sq.data() + 32768;
    // avgPower: channel-major sum over the padded SampleCount
    const int64_t nn = int64_t(SC) * ch;
    double avg = exact_seq_sum(
        nn, 0.0,
        [&](int64_t a, int64_t b, double* o) {
            int64_t j = a / SC, i = a - j * SC;
            for (int64_t k = a; k < b; ++k) {
                *o++ = SQ[pcm[size_t(i) * ch + size_t(j)]];
                if (++i == SC) {
                    i = 0;
                    ++j;
                }
            }
        },
        par, 8192, tm ? &st_avg : nullptr);
    avg = std::sqrt(avg / double(SC * ch));
    const auto q1 = now();
    // 1 - lerp(avgPower, smp, VariableFrameSizeRatio) per sample
    const double vfr = opt_.vfr;
    auto pw_of = [&](int64_t i) {
        double sm = 0.0;
        for (int j = 0; j < ch; ++j) sm += SQ[pcm[size_t(i) * ch + j]];
        sm = std::sqrt(sm / double(ch));
        return 1.0 - (avg + (sm - avg) * vfr);
    };
    std::vector<double, NoInitAlloc<double>> pw(static_cast<size_t>(SC));
    double* PW = pw.data();
    const double total = exact_seq_sum(
        SC, 0.0,
        [&](int64_t a, int64_t b, double* o) {  // pw is materialised on the way (the cut reads it)
            for (int64_t i = a; i < b; ++i) o[i - a] = PW[i] = pw_of(i);
        },
        par, 8192, tm ? &st_tot : nullptr);
    const double* P = PW;
    const auto q2 = now();
    const double per_frame = total / double(frame_count_est_);
    const auto q3 = now();
    // the cut: cur += pw[i]; at block-aligned i with cur >= perFramePower a frame
    // ends at i - 1 and cur restarts at 0 (pw[i] itself is not carried over)
    cut_frames(P, per_frame);
    file_first_ = {0, int(fr_start_.size())};  // one file
    if (tm)
        std::fprintf(stderr,
                     "plan [ms]: avg %.1f pw+total %.1f cut %.1f | exact sums: avg %lld/%lld blocks on the grid "
                     "(%lld ties), total %lld/%lld (%lld ties)\n",
                     ms(q0, q1), ms(q1, q2), ms(q3, now()), (long long)st_avg.fast_blocks, (long long)st_avg.blocks,
                     (long long)st_avg.ties, (long long)st_tot.fast_blocks, (long long)st_tot.blocks,
                     (long long)st_tot.ties);
    return 0;
}

void Encoder::cut_frames(const double* P, double per_frame) {
    const int SC = sample_count_, B = block_;
    // approximate prefix by 4096-sample blocks (speculation only)
    constexpr int kB = 4096;
    const int nb = (SC + kB - 1) / kB;
    std::vector<double> bsum(static_cast<size_t>(nb));
    parallel_for(nb, host_threads(), [&](int b) {
        double a = 0.0;
        const int i1 = std::min(SC, (b + 1) * kB);
        for (int i = b * kB; i < i1; ++i) a += P[i];
        bsum[size_t(b)] = a;
    });
    // approximate end of the frame whose running sum starts after `s` (frame 0: at 0)
    auto spec_end = [&](int first) -> int {  // first = first index added to cur
        double cur = 0.0;
        int i = first;
        while (i < SC) {
            const int b = i / kB;
            // skip whole blocks that cannot reach the threshold, even with +-1e-6 slack
            if (i == b * kB && b + 1 < nb && cur + bsum[size_t(b)] < per_frame * (1.0 - 1e-6) - 1e-6) {
                cur += bsum[size_t(b)];
                i = (b + 1) * kB;
                continue;
            }
            cur += P[i];
            if (i % B == 0 && cur >= per_frame) return i;
            ++i;
        }
        return SC;  // no cut: the last frame
    };
    // exact end (the reference's loop) of the frame whose sum starts at `first`
    auto exact_end = [&](int first) -> int {
        double cur = 0.0;
        for (int i = first; i < SC; ++i) {
            cur += P[i];
            if (i % B == 0 && cur >= per_frame) return i;
        }
        return SC;
    };
    std::vector<int> cuts;  // exact cut indices (frame k + 1 starts at cuts[k])
    int first = 0;          // frame 0 sums from 0, later frames from cut + 1
    for (;;) {
        // speculate the remaining cuts, then verify every frame's exact sum in parallel
        std::vector<int> spec;
        for (int f = first; f < SC;) {
            const int c = spec_end(f);
            if (c >= SC) break;
            spec.push_back(c);
            f = c + 1;
        }
        const int ns = int(spec.size());
        std::vector<int> exact(static_cast<size_t>(ns) + 1);
        parallel_for(ns + 1, host_threads(), [&](int k) {
            const int f = k == 0 ? first : spec[size_t(k - 1)] + 1;
            exact[size_t(k)] = f < SC ? exact_end(f) : SC;
        });
        int k = 0;
        while (k < ns && exact[size_t(k)] == spec[size_t(k)]) cuts.push_back(spec[size_t(k++)]);
        if (k == ns && exact[size_t(ns)] >= SC) break;  // every speculated frame verified, the last runs to the end
        // first mismatch: frame k's exact cut, then speculate again after it
        if (exact[size_t(k)] >= SC) break;
        cuts.push_back(exact[size_t(k)]);
        first = exact[size_t(k)] + 1;
        if (first >= SC) break;
    }
    fr_start_.clear();
    fr_end_.clear();
    int next = 0;
    for (int c : cuts) {
        fr_start_.push_back(next);
        fr_end_.push_back(c - 1);
        next = c;
    }
    fr_start_.push_back(next);
    fr_end_.push_back(SC - 1);
}

// TEncoder.Load + PrepareFrames (encoder.lpr:1111-1152, 1241-1273, 1294-1429)
int Encoder::prepare(const uint8_t* wav, size_t len, std::string* err) {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = load(wav, len, 0, INT64_MAX, err);
    if (rc != 0) return rc;
    const auto t1 = std::chrono::steady_clock::now();
    const int r2 = plan(err);
    if (std::getenv("GSC_HOST_TIMING")) {
        const auto t2 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "prepare [ms]: load %.1f plan %.1f (%d threads)\n",
                     std::chrono::duration<double, std::milli>(t1 - t0).count(),
                     std::chrono::duration<double, std::milli>(t2 - t1).count(), host_threads());
    }
    return r2;
}

int Encoder::prepare_many(const uint8_t* const* wavs, const size_t* lens, int nfiles, std::string* err) {
    if (nfiles <= 0) {
        *err = "prepare_many: no files";
        return -1;
    }
    std::vector<Encoder> es(static_cast<size_t>(nfiles), Encoder(opt_));
    for (int f = 0; f < nfiles; ++f) {
        const int rc = es[size_t(f)].prepare(wavs[f], lens[f], err);
        if (rc != 0) {
            *err = "file " + std::to_string(f) + ": " + *err;
            return rc;
        }
        const Encoder& a = es[size_t(f)];
        const Encoder& z = es[0];
        if (a.channels_ != z.channels_ || a.sample_rate_ != z.sample_rate_ ||
            a.opt_.chunks_per_frame != z.opt_.chunks_per_frame) {
            *err = "prepare_many: a batch needs one channel count, sample rate and ChunksPerFrame (file " +
                   std::to_string(f) + " differs)";
            return -2;
        }
    }
    *this = Encoder(es[0].opt_);
    channels_ = es[0].channels_;
    sample_rate_ = es[0].sample_rate_;
    block_ = es[0].block_;
    int64_t total = 0;
    for (const Encoder& a : es) total += a.sample_count_;
    if (total > INT32_MAX / 2) {
        *err = "prepare_many: batch too long";
        return -1;
    }
    sample_count_ = int(total);
    file_samples_ = sample_count_;
    pcm_off_ = 0;
    pcm_.resize(size_t(std::max<int64_t>(total, 1)) * size_t(channels_));
    file_first_.assign(1, 0);
    int64_t base = 0;
    for (const Encoder& a : es) {
        std::memcpy(pcm_.data() + size_t(base) * channels_, a.pcm_.data(), size_t(a.sample_count_) * channels_ * 2);
        for (size_t k = 0; k < a.fr_start_.size(); ++k) {
            fr_start_.push_back(int(base + a.fr_start_[k]));
            fr_end_.push_back(int(base + a.fr_end_[k]));
        }
        file_first_.push_back(int(fr_start_.size()));
        base += a.sample_count_;
    }
    return 0;
}

// an encoder over frame boundaries computed elsewhere (rank 0's PrepareFrames,
// multi-GPU sharding): the geometry of load(), then only the samples of frames
// [b, e) are copied
int Encoder::prepare_bounds(const uint8_t* wav, size_t len, const int* starts, const int* ends, int nframes, int b,
                            int e, std::string* err) {
    if (nframes <= 0 || b < 0 || e > nframes || b > e) {
        *err = "frame bounds: invalid frame range";
        return -1;
    }
    // geometry first (no samples), then validate the bounds against it
    int rc = load(wav, len, 0, 0, err);
    if (rc != 0) return rc;
    const int SC = sample_count_;
    if (starts[0] != 0 || ends[nframes - 1] != SC - 1) {
        *err = "frame bounds do not cover the file";
        return -1;
    }
    // frame 0 may be empty, (0, -1): the reference's cut ends it at i = 0 when
    // curPower >= perFramePower there (encoder.lpr:1411-1417; cut_frames keeps it)
    for (int i = 0; i < nframes; ++i)
        if (ends[i] < starts[i] - (i == 0 ? 1 : 0) || (i > 0 && starts[i] != ends[i - 1] + 1) ||
            starts[i] % block_ != 0) {
            *err = "frame bounds are not contiguous block-aligned frames";
            return -1;
        }
    fr_start_.assign(starts, starts + nframes);
    fr_end_.assign(ends, ends + nframes);
    file_first_ = {0, nframes};
    if (e > b) rc = load(wav, len, starts[b], int64_t(ends[e - 1]) + 1, err);
    return rc;
}

// MakeChunks srcData (encoder.lpr:467-485): chunk-major, channel-minor, zero
// past the frame end.  FindAttenuationDivider, the sign / reverse flags and
// the features run on the device (gsc_dsp.hip).
void Encoder::frame_host_src(FrameState& f) const {
    const int cs = opt_.chunk_size, ch = channels_;
    const int sc = f.sample_count;
    const int chunk_count = (sc - 1) / cs + 1;
    f.n = chunk_count * ch;
    f.neg.assign(size_t(f.n), 0);
    f.rev.assign(size_t(f.n), 0);
}

// chunk j's srcData (chunkRefs order: chunk-major, channel-minor; zero past
// the frame's samples), read from the loaded samples (encoder.lpr:467-485)
void Encoder::chunk_src(const FrameState& f, int j, double* out) const {
    const int cs = opt_.chunk_size, ch = channels_;
    const int i = j / ch, c = j - i * ch;
    const int16_t* base = pcm_.data() + (size_t(int64_t(f.start) - pcm_off_) * ch + size_t(c));
    for (int k = 0; k < cs; ++k) {
        const int pos = i * cs + k;
        out[k] = pos >= f.sample_count ? 0.0 : 0.0 + double(base[size_t(pos) * ch]) / 32767.0;  // srcData = s / 32767
    }
}

// TFrame.Reduce after the clustering (encoder.lpr:843-912)
void Encoder::frame_reduce_post(FrameState& f, bool reduced) const {
    const int cs = opt_.chunk_size, bd = opt_.chunk_bit_depth, D = 2 * cs;
    const double law = 1.0 / double(f.atten_div);
    const int obd = (1 << (bd - 1)) - 1;
    auto make_reduced = [&](int i, const double* rs) {
        double* dst = &f.rsrc[size_t(i) * cs];
        std::memcpy(dst, rs, sizeof(double) * cs);
        const int a = attenuation_of(hi_sample(dst, cs), law);
        bool ng, rv;
        sign_reverse(dst, cs, &ng, &rv);
        f.ratten[i] = uint8_t(a);
        f.rneg[i] = ng;
        const double cf = atten_coeff(a, law);
        for (int j = 0; j < cs; ++j) f.rdst[size_t(i) * cs + j] = output_sample(dst[j], obd, cf, ng);
    };
    if (reduced) {
        const int K = opt_.chunks_per_frame, N = f.n;
        std::vector<double> acc(size_t(K) * cs, 0.0);
        std::vector<int> count(size_t(K), 0);
        double s[16];
        for (int j = 0; j < N; ++j) {
            const int c = f.clusters[j];
            chunk_src(f, j, s);
            double* a = &acc[size_t(c) * cs];
            const double sg = f.neg[j] ? -1.0 : 1.0;
            for (int k = 0; k < cs; ++k) a[k] += s[f.rev[j] ? cs - 1 - k : k] * sg;
            ++count[c];
        }
        std::vector<int> order(static_cast<size_t>(K));
        for (int i = 0; i < K; ++i) order[i] = i;
        if (K > 1) fpc_quicksort(order.data(), count.data(), 0, K - 1);
        f.r = K;
        f.rsrc.assign(size_t(K) * cs, 0.0);
        f.rdst.assign(size_t(K) * cs, 0);
        f.ratten.assign(size_t(K), 0);
        f.rneg.assign(size_t(K), 0);
        double tmp[16];
        for (int i = 0; i < K; ++i) {
            const int id = order[i];
            const double y = double(count[id]);
            for (int j = 0; j < cs; ++j) {
                // div0 -> Single (encoder.lpr:863), nan0 (876)
                const double v = fpc::is_zero(y) ? 0.0 : acc[size_t(id) * cs + j] / y;
                const double sv = double(float(v));
                tmp[j] = std::isnan(sv) ? 0.0 : sv;
            }
            make_reduced(i, tmp);
        }
        (void)D;
    } else {
        const int N = f.n;
        f.r = N;
        f.rsrc.assign(size_t(N) * cs, 0.0);
        f.rdst.assign(size_t(N) * cs, 0);
        f.ratten.assign(size_t(N), 0);
        f.rneg.assign(size_t(N), 0);
        double s[16];
        for (int i = 0; i < N; ++i) {
            chunk_src(f, i, s);
            make_reduced(i, s);
        }
    }
}

// KNNFit post on the host (encoder.lpr:966-977): drop the entries no chunk
// uses, FPC QuickSort the survivors by use count, and reorder dstData and
// the attenuations.  remap[old] = new index (-1 for a dropped entry).  The
// per-chunk part (final index, dstNegative, dstReversed) and the index
// bitstream run on the device (gsc_pack.hip).
void Encoder::frame_prune(FrameState& f, const int* use, int* remap) const {
    const int cs = opt_.chunk_size;
    f.r_before_prune = f.r;
    std::vector<int> alive;
    alive.reserve(size_t(f.r));
    for (int i = 0; i < f.r; ++i) {
        remap[i] = -1;
        if (use[i] != 0) alive.push_back(i);
    }
    const int na = int(alive.size());
    std::vector<int> cnt(static_cast<size_t>(std::max(na, 1))), order(static_cast<size_t>(std::max(na, 1)));
    for (int i = 0; i < na; ++i) {
        cnt[i] = use[alive[i]];
        order[i] = i;
    }
    if (na > 1) fpc_quicksort(order.data(), cnt.data(), 0, na - 1);
    std::vector<int16_t> ndst(size_t(std::max(na, 1)) * cs);
    std::vector<uint8_t> natt(static_cast<size_t>(std::max(na, 1)));
    for (int i = 0; i < na; ++i) {
        const int o = alive[order[i]];
        remap[o] = i;
        std::memcpy(&ndst[size_t(i) * cs], &f.rdst[size_t(o) * cs], sizeof(int16_t) * cs);
        natt[i] = f.ratten[o];
    }
    f.rdst.swap(ndst);
    f.ratten.swap(natt);
    f.r = na;
}

// TFrame.SaveStream (encoder.lpr:980-1048) up to the band's chunk count:
// header, attenuations, dstData.  The index stream that follows
// (encoder.lpr:1050-1106) comes from the device packer.
void Encoder::frame_save_head(FrameState& f) const {
    const int cs = opt_.chunk_size, bd = opt_.chunk_bit_depth, ch = channels_;
    std::vector<uint8_t>& o = f.stream;
    o.clear();
    auto w8 = [&](unsigned v) { o.push_back(uint8_t(v)); };
    auto w16 = [&](unsigned v) {
        o.push_back(uint8_t(v));
        o.push_back(uint8_t(v >> 8));
    };
    auto w32 = [&](uint32_t v) {
        for (int i = 0; i < 4; ++i) o.push_back(uint8_t(v >> (8 * i)));
    };
    w16(unsigned((ch << 8) | 1));
    w16(unsigned(f.r));
    w16(unsigned((cs << 8) | bd));
    w32(uint32_t((opt_.chunk_blend << 24) | sample_rate_));
    w16(unsigned(f.atten_div));
    for (int j = 0; j < f.r / 2; ++j) w8(unsigned((f.ratten[2 * j] << 4) | f.ratten[2 * j + 1]));
    if (f.r & 1) w8(unsigned(f.ratten[f.r - 1] << 4));
    if (bd == 8) {
        for (size_t k = 0; k < size_t(f.r) * cs; ++k) w8(unsigned((f.rdst[k] + 128) & 0xff));
    } else {
        for (int j = 0; j < f.r; ++j) {
            const int16_t* d = &f.rdst[size_t(j) * cs];
            for (int k = 0; k < cs / 2; ++k) {
                const int s1 = d[2 * k] + 2048, s2 = d[2 * k + 1] + 2048;
                w8(unsigned(((s1 >> 4) & 0xf0) | ((s2 >> 8) & 0x0f)));
                w8(unsigned(s1 & 0xff));
                w8(unsigned(s2 & 0xff));
            }
            if (cs & 1) {
                const int s1 = d[cs - 1] + 2048;
                w8(unsigned((s1 >> 4) & 0xf0));
                w8(unsigned(s1 & 0xff));
            }
        }
    }
    w32(uint32_t(f.n / ch));
}

}  // namespace gsc
