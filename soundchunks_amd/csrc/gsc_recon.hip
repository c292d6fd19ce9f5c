// Reconstruction and PsyADelta on the device.
//
// After MakeFrames the reference rebuilds the 16-bit signal the .gsc encodes
// (encoder.lpr:2019-2027): TBand.MakeDstData (encoder.lpr:487-522) writes
// every final chunk's CS samples -- makeFloatSample of its reduced chunk,
// reversed and negated as KNNFit chose -- at the channel's running position,
// and TEncoder.MakeDstData (encoder.lpr:1518-1582) stores make16BitSample of
// the band sum.  With CBandCount = 1, underSample = 1 and ChunkBlend = 0 every
// output sample is written by exactly one chunk, so the whole reconstruction
// is one thread per (frame, chunk, sample): out = make16(0 + (0 + smp)).
// ComputePsyADelta (encoder.lpr:1862-1880) is sqrt(sum (src - dst)^2 / len)
// over Double copies of the SmallInt samples: every term and every partial
// sum is an integer, exact in f64 while the total stays below 2^53, so the
// sequential reference sum equals the exact integer sum the device reduces in
// any order (the host checks the bound and falls back to the sequential sum).
// f64 arithmetic here is the reference's (-ffp-contract=off: no FMA).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gsc_device.h"

namespace gsc {
namespace {

// make16BitSample (encoder.lpr:1638-1641): EnsureRange(round(smp * 32767)), round half to even
__device__ __forceinline__ int16_t make16(double smp) {
    double x = rint(smp * 32767.0);
    x = x < -32768.0 ? -32768.0 : (x > 32767.0 ? 32767.0 : x);
    return (int16_t)(int)x;
}

// makeFloatSample(smp, bd, atten, neg, law) (encoder.lpr:1665-1680)
__device__ __forceinline__ double make_float_sample(int16_t smp, int bd, int atten, bool neg, double law) {
    double coeff = 1.0;
    for (int i = 0; i <= atten; ++i) coeff += (double)i * law;
    const double obd = (double)((1 << (bd - 1)) - 1);
    const int16_t s16 = neg ? (int16_t)(-(int)smp) : smp;
    double r = (double)s16 / (obd * coeff);
    if (r < -1.0) r = -1.0;
    if (r > 1.0) r = 1.0;
    return r;
}

// grid: (ceil(max n*cs / 256), frames); out is interleaved [sample][channel]
__global__ __launch_bounds__(256) void recon_kernel(const ReconFrame* __restrict__ frames, int cs, int ch, int bd,
                                                    const uint32_t* __restrict__ chunk,
                                                    const int16_t* __restrict__ rdst,
                                                    const uint8_t* __restrict__ ratten, int16_t* __restrict__ out) {
    const ReconFrame f = frames[blockIdx.y];
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= (int64_t)f.n * cs) return;
    const int i = (int)(k / cs), j = (int)(k - (int64_t)i * cs);
    const int pos = (i / ch) * cs + j;  // the chunk's channel position (chunkRefs: chunk-major, channel-minor)
    if (pos >= f.sc) return;            // InRange(pos, 0, High(dstData[ch]))
    const uint32_t w = chunk[f.chunk_off + i];
    const int red = (int)(w >> 2);
    const bool neg = (w >> 1) & 1u, rev = w & 1u;
    const int16_t v = rdst[(f.red_off + red) * cs + (rev ? cs - 1 - j : j)];
    const double smp = make_float_sample(v, bd, ratten[f.red_off + red], neg, f.law);
    out[(f.out_off + pos) * ch + i % ch] = make16(0.0 + (0.0 + smp));
}

// sum over k < n of (a[k] - b[k])^2 as an exact integer
__global__ __launch_bounds__(256) void sqdiff_kernel(const int16_t* __restrict__ a, const int16_t* __restrict__ b,
                                                     int64_t n, unsigned long long* __restrict__ acc) {
    __shared__ unsigned long long part[4];
    unsigned long long s = 0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const long long d = (long long)a[k] - (long long)b[k];
        s += (unsigned long long)(d * d);
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(acc, part[0] + part[1] + part[2] + part[3]);
}

}  // namespace
}  // namespace gsc

using namespace gsc;

extern "C" hipError_t gsc_launch_recon(const ReconFrame* frames, int nframes, int max_n, int cs, int ch, int bd,
                                       const uint32_t* chunk, const int16_t* rdst, const uint8_t* ratten, int16_t* out,
                                       hipStream_t st) {
    if (nframes <= 0) return hipSuccess;
    const int64_t work = (int64_t)max_n * cs;
    const dim3 grid((unsigned)((work + 255) / 256), (unsigned)nframes), block(256);
    hipLaunchKernelGGL(recon_kernel, grid, block, 0, st, frames, cs, ch, bd, chunk, rdst, ratten, out);
    return hipGetLastError();
}

extern "C" hipError_t gsc_launch_sqdiff(const int16_t* a, const int16_t* b, int64_t n, unsigned long long* acc,
                                        hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t blocks = (n + 255) / 256;
    const unsigned grid = (unsigned)(blocks < 4096 ? blocks : 4096);
    hipLaunchKernelGGL(sqdiff_kernel, dim3(grid), dim3(256), 0, st, a, b, n, acc);
    return hipGetLastError();
}
