// Per-frame DSP of the encoder on the device: FindAttenuationDivider
// (encoder.lpr:566-605) and the chunk features of MakeChunks / TChunk
// ComputeDCT (encoder.lpr:258-322, 349-363, 467-485, 1700-1716).  f64
// throughout, in the reference's operation order (-ffp-contract=off, IEEE
// division and sqrt), so the results equal the host restatement in
// gsc_encoder.cpp bit for bit.
//
// Samples: one f64 row per channel (s / 32767, TEncoder.Load), row stride
// `span`.  Features land in the slab yakmo / KNNScanReduce read (X), so they
// never cross PCIe.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fpc_math.h"
#include "gsc_device.h"

namespace gsc {
namespace {

constexpr int kMaxAtt = 15;  // CMaxAttenuation (encoder.lpr:14)

__device__ __forceinline__ int64_t ceil_pos_d(double x) {  // FPC math.ceil, x >= 0
    const double t = trunc(x);
    int64_t r = (int64_t)t;
    if (x - t > 0.0) ++r;
    return r;
}

// the same for 0 <= x < 2^31 with the native f64 -> i32 conversion
__device__ __forceinline__ int ceil_pos_i32(double x) {
    const double t = trunc(x);
    int r = (int)t;
    if (x - t > 0.0) ++r;
    return r;
}

// FindAttenuationDivider: lane = candidate law 1/(lane+1); each lane runs the
// reference's sequential f64 error sum over (channel, chunk, sample), then the
// first lane at the minimum wins (strict <, laws in order).
//
// One workgroup of 8 waves per frame.  The error terms (x - r)^2 of a batch
// of kAttBatch samples are independent across samples: seven producer waves
// compute them (chunk c of the batch on wave 1 + c % 7, lane = law) into LDS,
// and wave 0 adds them in the reference's order while the producers fill the
// other buffer.  Every term is the reference's own arithmetic, and the sum is
// the same sequential chain, so the result is unchanged; the f64 latency
// chains now run on all four SIMDs instead of one.
constexpr int kAttProd = 7;                  // producer waves
constexpr int kAttBatchMax = kAttProd * 16;  // samples per batch (LDS: two buffers of 64 lanes x f64)
constexpr int kAttThreads = 64 * (kAttProd + 1);
// samples per batch for a ChunkSize: whole chunks, the same number per producer
__host__ __device__ constexpr int att_batch(int cs) { return kAttProd * cs * (cs >= 16 ? 1 : 16 / cs); }

template <int CS>
__global__ __launch_bounds__(kAttThreads) void atten_kernel(DspFrame* __restrict__ frames, int nframes,
                                                            const double* __restrict__ samp, int64_t span, int ch,
                                                            int obd) {
    constexpr int kAttBatch = att_batch(CS);
    static_assert(kAttBatch % (CS * kAttProd) == 0 && kAttBatch <= kAttBatchMax, "whole chunks per producer");
    extern __shared__ __attribute__((aligned(16))) double aterm[];  // [2][kAttBatch][64]
    const int fi = blockIdx.x;
    if (fi >= nframes) return;
    DspFrame* fr = frames + fi;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double law = 1.0 / double(lane + 1);
    // coeff(a) = 1 + sum_{i=0..a} i*law, left to right (encoder.lpr:1654-1656)
    double coeff[kMaxAtt + 1];
    {
        double c = 1.0;
#pragma unroll
        for (int a = 0; a <= kMaxAtt; ++a) {
            c += double(a) * law;
            coeff[a] = c;
        }
    }
    const int sc = fr->sc, nck = sc / CS;
    const int tot = nck * CS;  // samples of whole chunks per channel
    const int nbat = (tot + kAttBatch - 1) / kAttBatch;
    const double dobd = double(obd);
    double v = 0.0;
    for (int j = 0; j < ch; ++j) {
        const double* src = samp + int64_t(j) * span + fr->s_off;
        for (int t = 0; t <= nbat; ++t) {
            if (wave > 0 && t < nbat) {
                // terms of batch t into buffer t & 1
                double* T = aterm + size_t(t & 1) * kAttBatch * 64;
                const int t0 = t * kAttBatch;
                const int kn = min(kAttBatch, tot - t0) / CS;
                for (int k = wave - 1; k < kn; k += kAttProd) {
                    double x[CS];
#pragma unroll
                    for (int l = 0; l < CS; ++l) x[l] = src[t0 + k * CS + l];
                    // hiSmp (encoder.lpr:1687-1689); |x| <= 32768/32767, so every value
                    // here fits an int32 and the native conversions are exact
                    int hi = 0;
#pragma unroll
                    for (int l = 0; l < CS; ++l) {
                        const int h = ceil_pos_i32(fabs(x[l] * 32767.0));
                        hi = h > hi ? h : hi;
                    }
                    // ComputeAttenuation (encoder.lpr:1691-1697): coeff after r steps = coeff[r]
                    int a = kMaxAtt;
                    for (int r = 1; r <= kMaxAtt; ++r)
                        if (double(hi) * coeff[r] > 32767.0) {
                            a = r - 1;
                            break;
                        }
                    double cf = coeff[0];
#pragma unroll
                    for (int q = 1; q <= kMaxAtt; ++q) cf = q == a ? coeff[q] : cf;
                    const double den = dobd * cf;
#pragma unroll
                    for (int l = 0; l < CS; ++l) {
                        // makeOutputSample (encoder.lpr:1648-1663): Round, SmallInt wrap, clamp
                        // (|x obd cf| <= 1.00003 * 32767 * 121 < 2^22: the i32 conversion is exact)
                        int s16 = (int)(int16_t)(int)rint(x[l] * dobd * cf);
                        s16 = max(s16, -obd + 1);
                        s16 = min(s16, obd - 1);
                        // makeFloatSample (encoder.lpr:1665-1680)
                        double r = double(s16) / den;
                        r = r < -1.0 ? -1.0 : r;
                        r = r > 1.0 ? 1.0 : r;
                        const double dd = x[l] - r;
                        T[(k * CS + l) * 64 + lane] = dd * dd;
                    }
                }
            }
            if (wave == 0 && t > 0) {
                // the reference's sum over batch t - 1, in sample order
                const double* T = aterm + size_t((t - 1) & 1) * kAttBatch * 64;
                const int n = min(kAttBatch, tot - (t - 1) * kAttBatch);
                for (int q = 0; q < n; ++q) v += T[q * 64 + lane];
            }
            __syncthreads();
        }
    }
    if (wave != 0) return;
    // first lane at the minimum (best starts at MaxSingle, v < best)
    double best = v;
    int bi = lane;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double ov = __shfl_xor(best, o);
        const int oi = __shfl_xor(bi, o);
        if (ov < best || (ov == best && oi < bi)) {
            best = ov;
            bi = oi;
        }
    }
    if (lane == 0) fr->atten_div = best < 3.4028234663852886e+38 ? bi + 1 : 1;
}

struct Trig {
    double dct[16 * 16], dft_c[16 * 16], dft_s[16 * 16], idft_c[16 * 16], idft_s[16 * 16];
};

// one chunk per thread: srcData, sign / reverse heuristics, DCT-II, cepstrum
template <int CS>
__global__ __launch_bounds__(256) void features_kernel(const DspFrame* __restrict__ frames, int nframes,
                                                       const double* __restrict__ samp, int64_t span, int ch,
                                                       const double* __restrict__ trig_g, double s0, double scale,
                                                       float* __restrict__ X, uint8_t* __restrict__ nr,
                                                       float* __restrict__ Q) {
    __shared__ double tr[5 * CS * CS];
    for (int i = threadIdx.x; i < 5 * CS * CS; i += blockDim.x) tr[i] = trig_g[i];
    __syncthreads();
    const double* dct = tr;
    const double* dft_c = tr + CS * CS;
    const double* dft_s = tr + 2 * CS * CS;
    const double* idft_c = tr + 3 * CS * CS;
    const double* idft_s = tr + 4 * CS * CS;
    const int fi = blockIdx.y;
    if (fi >= nframes) return;
    const DspFrame fr = frames[fi];
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= fr.n) return;
    constexpr int DP = feature_stride(CS);  // slab row: 2*CS features, then zeros
    const int i = c / ch, j = c - i * ch;
    // chunk samples, zero past the frame end (encoder.lpr:467-485: 0 + sample)
    double s[CS];
    const double* row = samp + int64_t(j) * span + fr.s_off;
#pragma unroll
    for (int k = 0; k < CS; ++k) {
        const int pos = i * CS + k;
        s[k] = pos >= fr.sc ? 0.0 : 0.0 + row[pos];
    }
    // TChunk.ComputeDstAttributes sign / reverse (encoder.lpr:374-396)
    double p1 = 0.0, p2 = 0.0;
#pragma unroll
    for (int k = 0; k < CS; ++k)
        if (s[k] < 0) p1 -= s[k];
#pragma unroll
    for (int k = 0; k < CS; ++k)
        if (s[k] > 0) p2 += s[k];
    const bool neg = p1 > p2;
    p1 = 0.0;
    p2 = 0.0;
#pragma unroll
    for (int k = 0; k < CS / 2; ++k) p1 += fabs(s[k]);
#pragma unroll
    for (int k = CS / 2; k < CS; ++k) p2 += fabs(s[k]);
    const bool rev = p1 > p2;
    nr[fr.c_off + c] = (uint8_t)((neg ? 1 : 0) | (rev ? 2 : 0));
    if (Q) {  // KNNFit queries: Single(srcData) (encoder.lpr:945-948)
        float* qo = Q + (fr.c_off + c) * CS;
#pragma unroll
        for (int k = 0; k < CS; ++k) qo[k] = float(s[k]);
    }
    double data[CS], temp[CS];
#pragma unroll
    for (int k = 0; k < CS; ++k) data[k] = s[rev ? CS - 1 - k : k] * (neg ? -1.0 : 1.0);
    float* out = X + fr.x_off + int64_t(c) * DP;
#pragma unroll
    for (int k = 2 * CS; k < DP; ++k) out[k] = 0.0f;
    // DCT-II (encoder.lpr:258-276)
#pragma unroll
    for (int k = 0; k < CS; ++k) {
        const double sk = k == 0 ? s0 : 1.0;
        double sum = 0.0;
#pragma unroll
        for (int n = 0; n < CS; ++n) sum += sk * data[n] * dct[k * CS + n];
        out[k] = float(sum * scale);
    }
    // power spectrum, log10, inverse DFT magnitude * 1e-5 (encoder.lpr:278-322, 1700-1716)
#pragma unroll
    for (int k = 0; k < CS; ++k) {
        double re = 0.0, im = 0.0;
#pragma unroll
        for (int q = 0; q < CS; ++q) {
            re += data[q] * dft_c[k * CS + q];
            im += data[q] * dft_s[k * CS + q];
        }
        temp[k] = re * re + im * im;
    }
#pragma unroll
    for (int k = 0; k < CS; ++k)
        if (!fpc::is_zero(temp[k])) temp[k] = fpc::log10(temp[k]);
#pragma unroll
    for (int k = 0; k < CS; ++k) {
        double re = 0.0, im = 0.0;
#pragma unroll
        for (int q = 0; q < CS; ++q) {
            re += temp[q] * idft_c[k * CS + q];
            im += temp[q] * idft_s[k * CS + q];
        }
        re /= double(CS);
        im /= double(CS);
        out[CS + k] = float(__dsqrt_rn(re * re + im * im) * 0.00001);
    }
}

// TEncoder.Load's sample conversion (encoder.lpr:1111-1152): SmallInt / 32767
// into the planar f64 slab the DSP kernels read; pcm = [sample][ch] of the span
__global__ __launch_bounds__(256) void pcm_kernel(const int16_t* __restrict__ pcm, int64_t span, int ch,
                                                  double* __restrict__ samp) {
    const int64_t total = span * ch;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = p / ch;
        const int j = (int)(p - t * ch);
        samp[(int64_t)j * span + t] = (double)pcm[p] / 32767.0;
    }
}

}  // namespace
}  // namespace gsc

using namespace gsc;

extern "C" hipError_t gsc_launch_pcm(const int16_t* pcm, int64_t span, int ch, double* samp, hipStream_t st) {
    const int64_t total = span * ch;
    if (total <= 0) return hipSuccess;  // an empty span (a frame (0, -1): encoder.lpr:1411-1417)
    const int64_t blocks = (total + 255) / 256;
    hipLaunchKernelGGL(pcm_kernel, dim3((unsigned)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, st, pcm, span, ch,
                       samp);
    return hipGetLastError();
}

// FindAttenuationDivider for every frame (one 8-wave workgroup per frame)
extern "C" hipError_t gsc_launch_atten(int cs, DspFrame* frames, int nframes, const double* samp, int64_t span, int ch,
                                       int obd, hipStream_t st) {
    const size_t shm = size_t(2) * att_batch(cs) * 64 * sizeof(double);
    switch (cs) {
#define AK(CSV)                                                                                                  \
    case CSV:                                                                                                    \
        if (hipError_t e = hipFuncSetAttribute((const void*)atten_kernel<CSV>,                                   \
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm))            \
            return e;                                                                                            \
        hipLaunchKernelGGL(atten_kernel<CSV>, dim3(nframes), dim3(kAttThreads), shm, st, frames, nframes, samp,  \
                           span, ch, obd);                                                                       \
        break;
        AK(1) AK(2) AK(3) AK(4) AK(5) AK(6) AK(7) AK(8) AK(9) AK(10) AK(11) AK(12) AK(13) AK(14) AK(15) AK(16)
#undef AK
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// chunk features for every frame (slab rows of feature_stride(CS) floats); trig = 5 CS x CS f64 tables
// (dct, dft cos/sin, idft cos/sin)
extern "C" hipError_t gsc_launch_features(int cs, const DspFrame* frames, int nframes, int max_n, const double* samp,
                                          int64_t span, int ch, const double* trig, double s0, double scale, float* X,
                                          uint8_t* nr, float* Q, hipStream_t st) {
    if (max_n <= 0 || nframes <= 0) return hipSuccess;
    const dim3 grid((max_n + 255) / 256, nframes), block(256);
    switch (cs) {
#define FK(CSV)                                                                                                  \
    case CSV:                                                                                                    \
        hipLaunchKernelGGL(features_kernel<CSV>, grid, block, 0, st, frames, nframes, samp, span, ch, trig, s0,   \
                           scale, X, nr, Q);                                                                     \
        break;
        FK(1) FK(2) FK(3) FK(4) FK(5) FK(6) FK(7) FK(8) FK(9) FK(10) FK(11) FK(12) FK(13) FK(14) FK(15) FK(16)
#undef FK
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
