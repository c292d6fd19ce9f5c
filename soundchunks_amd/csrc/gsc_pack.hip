// TFrame.KNNFit post-processing and TFrame.SaveStream's chunk-index
// bitstream on MI355X (gfx950): SURVEY.md §8 f2.
//
//   usecount_kernel  per-entry use counts of KNNFit's choices
//                    (reducedChunks[i].useCount, encoder.lpr:966-970); the host
//                    prunes unused entries and runs the FPC QuickSort by count
//                    (encoder.lpr:970-977) on these K counts and uploads the
//                    resulting old -> new index map
//   pack_kernel      SaveStream's variable-length index codes
//                    (encoder.lpr:1050-1106) as a parallel prefix-sum packer
//
// The reference packs sequentially into a 32-bit `bits` register, flushing a
// 16-bit word whenever bitCnt >= 16.  With CMaxChunksPerFrame = 4096
// (encoder.lpr:15, -cpf is clamped to it at :1993) an index has at most 12
// bits, so vcbsCnt <= 3 and a code is at most 2 + 3 + 12 = 17 bits.  A 17-bit
// code needs a vcbsCnt change to 3, so the code after it has at most 15 bits
// (same vcbsCnt: 2 + 1 + 12) or 14 (a change back); bitCnt + codeSize
// therefore never exceeds 32 and no code bit is ever shifted out of `bits`.
// The stream is then exactly the LSB-first concatenation of the codes,
// written as little-endian 16-bit words, the last one zero-padded: code j
// starts at bit offset sum_{i<j} size_i, which is an exclusive prefix sum.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gsc_device.h"

namespace gsc {

constexpr int kPackThreads = 1024;
constexpr int kPackPerThread = 8;  // consecutive chunks per thread per tile

// vcbsCnt of a reduced-chunk index (encoder.lpr:1054): 0 for index 0, else
// BsrWord(index) div CVariableCodingBlockSize
__device__ __forceinline__ int vc_of(int idx) { return idx == 0 ? 0 : (31 - __clz(idx)) / 3; }

__global__ __launch_bounds__(1024) void usecount_kernel(const PackFrame* __restrict__ frames,
                                                        const int* __restrict__ best, int* __restrict__ counts) {
    __shared__ int h[kMaxK];
    const PackFrame& f = frames[blockIdx.x];
    const int N = f.N, R = f.R;
    const int* b = best + f.out_off;
    int* c = counts + f.r_off;
    if (R > kMaxK) {
        // -pr0 passthrough frames: reducedChunks = every chunk (encoder.lpr:891-905),
        // more entries than the LDS histogram holds; count in the frame's slab
        for (int i = threadIdx.x; i < R; i += blockDim.x) c[i] = 0;
        __syncthreads();
        for (int j = threadIdx.x; j < N; j += blockDim.x) {
            const int v = b[j];
            if (v >= 0) atomicAdd(&c[v >> 2], 1);
        }
        return;
    }
    for (int i = threadIdx.x; i < R; i += blockDim.x) h[i] = 0;
    __syncthreads();
    for (int j = threadIdx.x; j < N; j += blockDim.x) {
        const int v = b[j];
        if (v >= 0) atomicAdd(&h[v >> 2], 1);  // -1: a tie-overflow query awaiting the ANN replay
    }
    __syncthreads();
    for (int i = threadIdx.x; i < R; i += blockDim.x) c[i] = h[i];
}

// One workgroup per frame.  Chunk j's reduced index is remap[best[j] >> 2]
// (the pruned, count-sorted order), dstNegative = best bit 1, dstReversed =
// best bit 0 (encoder.lpr:960-964).  Tiles of 8192 chunks: sizes, a block
// exclusive scan, then every code is OR-ed into the zeroed word slab at its
// bit offset (a code straddles at most two 32-bit words).
__global__ __launch_bounds__(kPackThreads) void pack_kernel(PackFrame* __restrict__ frames, const int* __restrict__ best,
                                                            const int* __restrict__ remap, uint32_t* __restrict__ words,
                                                            uint32_t* __restrict__ codes_out) {
    __shared__ int wsum[kPackThreads / 64];
    __shared__ int carry;
    __shared__ int overrun;
    PackFrame& f = frames[blockIdx.x];
    const int N = f.N;
    const int* b = best + f.out_off;
    const int* rm = remap + f.r_off;
    uint32_t* w = words + f.w_off;
    // the slab's capacity: a code that would land past it is not written and
    // the frame reports nbits = -1 (the 17-bit premise above broke), so a
    // broken premise can never corrupt the next frame's slab
    const int64_t cap = (int64_t(N) * 17 + 31) / 32 + 1;  // pack_word_capacity(N)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) {
        carry = 0;
        overrun = 0;
    }
    __syncthreads();
    for (int base = 0; base < N; base += kPackThreads * kPackPerThread) {
        const int j0 = base + tid * kPackPerThread;
        uint32_t code[kPackPerThread];
        int size[kPackPerThread];
        int prev = -1;  // prevVcbsCnt (encoder.lpr:1058-1060)
        if (j0 >= 1 && j0 - 1 < N) prev = vc_of(rm[b[j0 - 1] >> 2]);
        int sum = 0;
#pragma unroll
        for (int e = 0; e < kPackPerThread; ++e) {
            const int j = j0 + e;
            code[e] = 0;
            size[e] = 0;
            if (j < N) {
                const int v = b[j];
                const int idx = rm[v >> 2];
                const int vc = vc_of(idx);
                uint32_t c = uint32_t((v >> 1) & 1) | (uint32_t(v & 1) << 1);  // dstNegative, dstReversed
                int s = 2;
                if (vc == prev) {
                    s += 1;
                } else {
                    c |= 1u << s;
                    s += 1;
                    c |= uint32_t(vc) << s;
                    s += 2;  // CVariableCodingHeaderSize
                }
                for (int k = vc; k >= 0; --k) {
                    c |= uint32_t((idx >> (3 * k)) & 7) << s;
                    s += 3;  // CVariableCodingBlockSize
                }
                code[e] = c;
                size[e] = s;
                sum += s;
                prev = vc;
                if (codes_out) codes_out[f.out_off + j] = uint32_t(idx) << 2 | uint32_t(v & 3);
            }
        }
        // block exclusive scan of the per-thread bit counts
        int incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o, 64);
            if (lane >= o) incl += t;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        int wbase = 0;
        for (int i = 0; i < wave; ++i) wbase += wsum[i];
        int total = 0;
        for (int i = 0; i < kPackThreads / 64; ++i) total += wsum[i];
        int bit = carry + wbase + incl - sum;
#pragma unroll
        for (int e = 0; e < kPackPerThread; ++e) {
            if (size[e] == 0) continue;
            const int wi = bit >> 5, sh = bit & 31;
            const bool two = sh + size[e] > 32;
            if (wi + (two ? 1 : 0) >= cap) {
                overrun = 1;
            } else {
                atomicOr(&w[wi], code[e] << sh);
                if (two) atomicOr(&w[wi + 1], code[e] >> (32 - sh));
            }
            bit += size[e];
        }
        __syncthreads();  // everyone has read carry and wsum
        if (tid == 0) carry += total;
        __syncthreads();
    }
    __syncthreads();
    if (tid == 0) f.nbits = overrun ? -1 : carry;
}

}  // namespace gsc

using namespace gsc;

// counts: R ints per frame at r_off (overwritten)
extern "C" hipError_t gsc_launch_usecount(const PackFrame* frames, int nframes, const int* best, int* counts,
                                          hipStream_t st) {
    if (nframes <= 0) return hipSuccess;
    hipLaunchKernelGGL(usecount_kernel, dim3(nframes), dim3(1024), 0, st, frames, best, counts);
    return hipGetLastError();
}

// words: the frames' slabs (capacity pack_word_capacity(N) each) must be zeroed;
// codes (optional): N words per frame at out_off, final index << 2 | neg << 1 | rev
extern "C" hipError_t gsc_launch_pack(PackFrame* frames, int nframes, const int* best, const int* remap,
                                      uint32_t* words, uint32_t* codes, hipStream_t st) {
    if (nframes <= 0) return hipSuccess;
    hipLaunchKernelGGL(pack_kernel, dim3(nframes), dim3(kPackThreads), 0, st, frames, best, remap, words, codes);
    return hipGetLastError();
}
