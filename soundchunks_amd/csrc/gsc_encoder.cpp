// Host stages of the encoder (see gsc_encoder.h).  Each function cites the
// reference encoder/encoder.lpr lines it reproduces bit-exactly.
#include "gsc_encoder.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "fpc_math.h"

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

// TEncoder.Load + PrepareFrames (encoder.lpr:1111-1152, 1241-1273, 1294-1429)
int Encoder::prepare(const uint8_t* wav, size_t len, std::string* err) {
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
    if (!(o.chunk_size == 4 || o.chunk_size == 8 || o.chunk_size == 16)) {
        *err = "ChunkSize must be 4, 8 or 16";
        return -2;
    }
    const int cs = o.chunk_size, ch = channels_;
    const int sc = int((len - 44) / (2 * size_t(ch)));
    const double hc = std::min(o.high_cut, double(sample_rate_) / 2);
    const double fcl = o.low_cut / double(sample_rate_), fch = hc / double(sample_rate_);
    if (fcl > 0.0 || fch < 0.5) {
        *err = "band-pass filtering (-lc/-hc below Nyquist) is not supported";
        return -2;
    }
    const int under = int(std::max<int64_t>(1, fpc::round(0.25 / fch)));
    block_ = under * (cs - o.chunk_blend);
    sample_count_ = ((sc - 1) / block_ + 1) * block_;  // Pascal div truncates
    const int SC = sample_count_;
    filtered_.resize(size_t(ch));
    for (auto& v : filtered_) v.resize(size_t(std::max(SC, 1)));  // no fill: the workers below write every sample
    pcm_.resize(size_t(std::max(SC, 1)) * size_t(ch));
    const uint8_t* d = wav + 44;
    // per-sample work in parallel blocks; every sequential f64 sum below keeps
    // the reference's order (encoder.lpr:1374-1425)
    constexpr int kBlk = 1 << 16;
    const int nblk = (std::max({SC, sc, 1}) + kBlk - 1) / kBlk;
    parallel_for(nblk, host_threads(), [&](int k) {
        const int i1 = std::min(sc, (k + 1) * kBlk);
        for (int i = k * kBlk; i < i1; ++i)
            for (int c = 0; c < ch; ++c) {
                const uint8_t* b = d + (size_t(i) * ch + c) * 2;
                const int16_t v = int16_t(uint16_t(b[0] | (b[1] << 8)));
                pcm_[size_t(i) * ch + c] = v;
                filtered_[c][i] = double(v) / 32767.0;
            }
        const int z1 = std::min(std::max(SC, 1), (k + 1) * kBlk);  // zero padding past the WAV end
        for (int i = std::max(sc, k * kBlk); i < z1; ++i)
            for (int c = 0; c < ch; ++c) {
                pcm_[size_t(i) * ch + c] = 0;
                filtered_[c][i] = 0.0;
            }
    });
    const int frame_count = int(fpc::ceil_pos(double(SC) / (double(sample_rate_) * (o.frame_length / 1000.0))));
    // ChunksPerFrame search only changes anything with -br (encoder.lpr:1337-1351)
    int cpf = o.chunks_per_frame;
    if (o.bit_rate > 0) {
        const long long projected =
            (long long)std::ceil((double(SC) / double(sample_rate_)) * (double(o.bit_rate) * 1024.0 / 8.0));
        ++cpf;
        for (;;) {
            --cpf;
            const double band = (double(SC) * double(ch) * (std::log2(double(cpf)) + 3 + 1 + 1)) /
                                (8.0 * double(cs - o.chunk_blend) * double(under));
            const double frame = double(cpf * cs) * double(o.chunk_bit_depth) / 8.0 + double(cpf) * 4.0 / 8.0 + 16;
            const int32_t tent = int32_t(fpc::round(0.0 + band * 0.8 + double(frame_count) * frame));
            if (tent <= projected || cpf <= 1) break;
        }
        opt_.chunks_per_frame = cpf;
    }
    // pass 2: RMS-power balanced frame boundaries, sequential f64 (encoder.lpr:1374-1425)
    double avg = 0.0;
    for (int j = 0; j < ch; ++j) {
        const double* f = filtered_[j].data();
        for (int i = 0; i < SC; ++i) avg += f[i] * f[i];
    }
    avg = std::sqrt(avg / double(SC * ch));
    std::vector<double> pw(static_cast<size_t>(std::max(SC, 1)));
    parallel_for(nblk, host_threads(), [&](int k) {
        const int i1 = std::min(SC, (k + 1) * kBlk);
        for (int i = k * kBlk; i < i1; ++i) {
            double s = 0.0;
            for (int j = 0; j < ch; ++j) s += filtered_[j][i] * filtered_[j][i];
            s = std::sqrt(s / double(ch));
            pw[i] = 1.0 - (avg + (s - avg) * o.vfr);
        }
    });
    double total = 0.0;
    for (int i = 0; i < SC; ++i) total += pw[i];
    const double per_frame = total / double(frame_count);
    fr_start_.clear();
    fr_end_.clear();
    int next = 0;
    double cur = 0.0;
    for (int i = 0, r = 0; i < SC; ++i, r = (r + 1 == block_) ? 0 : r + 1) {  // r = i mod block_
        cur += pw[i];
        if ((r == 0) && (cur >= per_frame)) {
            fr_start_.push_back(next);
            fr_end_.push_back(i - 1);
            cur = 0.0;
            next = i;
        }
    }
    fr_start_.push_back(next);
    fr_end_.push_back(SC - 1);
    return 0;
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
    const double* row = filtered_[size_t(c)].data() + f.start;
    for (int k = 0; k < cs; ++k) {
        const int pos = i * cs + k;
        out[k] = pos >= f.sample_count ? 0.0 : 0.0 + row[pos];
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
