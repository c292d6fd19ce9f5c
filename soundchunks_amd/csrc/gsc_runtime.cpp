// MI355X runtime for the SoundChunks hot path: device selection, HBM slabs,
// batched launches of the Reduce (yakmo + KNNScanReduce) and KNNFit kernels
// over many frames at once, host thread pool for the per-frame DSP, and the
// C ABI declared in include/soundchunks.h.
#include <cstddef>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <new>
#include <string>
#include <strings.h>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/soundchunks.h"
#include "fpc_math.h"
#include "gsc_device.h"
#include "gsc_encoder.h"

extern "C" hipError_t gsc_launch_yakmo(int D, const gsc::ReduceFrame* frames, int nframes, const float* X, float* C,
                                       float* fs, int* is, float* gsum, uint32_t* gbits, int max_n, hipStream_t st);
extern "C" size_t gsc_yakmo_big_floats(int64_t total_points, int nframes);
extern "C" size_t gsc_yakmo_big_words(int64_t total_points, int nframes);
extern "C" int gsc_yakmo_max_lds_points(void);
extern "C" hipError_t gsc_launch_scan_pass(int D, gsc::ReduceFrame* frames, int nframes, int K, const float* X,
                                           float* C, int* is, float* fs, const float* rate_tab, double tol, int max_passes,
                                           int only_flagged, hipStream_t st);
extern "C" hipError_t gsc_launch_scan_batch(int D, int logk, gsc::ReduceFrame* frames, int nframes, const float* X,
                                            float* C, int* is, const float* rate_tab, double tol, int max_passes,
                                            int opts, float* tails, hipStream_t st);
extern "C" size_t gsc_scan_tail_floats_per_frame(int D, int logk);
extern "C" hipError_t gsc_launch_atten(int cs, gsc::DspFrame* frames, int nframes, const double* samp, int64_t span,
                                       int ch, int obd, hipStream_t st);
extern "C" hipError_t gsc_launch_features(int cs, const gsc::DspFrame* frames, int nframes, int max_n,
                                          const double* samp, int64_t span, int ch, const double* trig, double s0,
                                          double scale, float* X, uint8_t* nr, float* Q, hipStream_t st);
extern "C" hipError_t gsc_launch_pcm(const int16_t* pcm, int64_t span, int ch, double* samp, hipStream_t st);
extern "C" hipError_t gsc_launch_knnfit(int CS, gsc::FitFrame* frames, int nframes, int max_n, int max_r,
                                        const float* cand, const float* q, int* out, hipStream_t st);
extern "C" hipError_t gsc_launch_recon(const gsc::ReconFrame* frames, int nframes, int max_n, int cs, int ch, int bd,
                                       const uint32_t* chunk, const int16_t* rdst, const uint8_t* ratten, int16_t* out,
                                       hipStream_t st);
extern "C" hipError_t gsc_launch_sqdiff(const int16_t* a, const int16_t* b, int64_t n, unsigned long long* acc,
                                        hipStream_t st);
extern "C" hipError_t gsc_launch_usecount(const gsc::PackFrame* frames, int nframes, const int* best, int* counts,
                                          hipStream_t st);
extern "C" hipError_t gsc_launch_pack(gsc::PackFrame* frames, int nframes, const int* best, const int* remap,
                                      uint32_t* words, uint32_t* codes, hipStream_t st);
extern "C" hipError_t gsc_launch_ann_build_many(const void* trees, int ntrees, hipStream_t st);
extern "C" hipError_t gsc_launch_knnfit_ann(const void* trees, const void* jobs, int njobs, const float* q, int* out,
                                            float* pq_key, void* pq_node, int pq_cap, hipStream_t st);

namespace gsc {

void parallel_for(int n, int threads, const std::function<void(int)>& fn) {
    if (threads <= 1 || n <= 1) {
        for (int i = 0; i < n; ++i) fn(i);
        return;
    }
    std::atomic<int> next{0};
    std::vector<std::thread> pool;
    const int t = std::min(threads, n);
    pool.reserve(size_t(t));
    for (int k = 0; k < t; ++k)
        pool.emplace_back([&] {
            for (;;) {
                const int i = next.fetch_add(1);
                if (i >= n) break;
                fn(i);
            }
        });
    for (auto& th : pool) th.join();
}

int host_threads() {
    static int n = [] {
        const char* e = std::getenv("GSC_HOST_THREADS");
        if (e && std::atoi(e) > 0) return std::atoi(e);
        const unsigned hc = std::thread::hardware_concurrency();
        return int(std::min(16u, std::max(1u, hc)));
    }();
    return n;
}

namespace {

thread_local std::string t_err;
thread_local gsc_timing t_tim;

int fail(const std::string& m) {
    t_err = m;
    return -1;
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) return fail(std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// The hot path requires a gfx950 device; there is no CPU fallback.
int ensure_device() {
    static int state = 0;  // 0 unknown, 1 ok, -1 bad
    static std::string why;
    if (state == 0) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
            why = "no HIP device visible (the MI355X hot path has no CPU fallback)";
            state = -1;
        } else {
            hipDeviceProp_t p;
            int dev = 0;
            if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) {
                why = "cannot query the HIP device";
                state = -1;
            } else if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0) {
                why = std::string("device is ") + p.gcnArchName + ", kernels are built for gfx950 only";
                state = -1;
            } else {
                state = 1;
            }
        }
    }
    if (state < 0) return fail(why);
    (void)hipGetLastError();  // a failure of an earlier unrelated call must not fail this one's launch checks
    return 0;
}

// diagnostic (GSC_HOST_TIMING): host time inside hipMalloc / hipFree of DevBufs
std::atomic<int64_t> g_devbuf_ns{0};

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    ~DevBuf() {
        if (p) {
            const double t = now_ms();
            (void)hipFree(p);
            g_devbuf_ns.fetch_add(int64_t((now_ms() - t) * 1e6));
        }
    }
    hipError_t alloc(size_t count) {
        n = count;
        const double t = now_ms();
        const hipError_t e = hipMalloc(&p, sizeof(T) * std::max<size_t>(count, 1));
        g_devbuf_ns.fetch_add(int64_t((now_ms() - t) * 1e6));
        return e;
    }
};

// Device scratch of the KNNFit overflow replay: one grow-only hipMalloc
// block carved into aligned sub-buffers, owned by the caller (the encode's
// PostCtx, or the synchronous drop-in call) and freed only when the caller is
// done.  Round 4 ran the replay on stream-ordered pool memory
// (hipMallocAsync / hipFreeAsync); a second replay in one process faulted on
// the null stream, and the workaround there (plain hipMalloc) left the pool
// path in the encoder.  The arena replaces both: no pool, no free while a
// replay can still be in flight (hipFree of a retired block waits for the
// device, so retired blocks are kept until the owner is destroyed), and every
// sub-buffer is poison-filled (0xff bytes: NaN floats, -1 ints) before each
// replay, so a read of memory the replay did not write cannot hide behind the
// zero pages a fresh hipMalloc returns -- the GPU tests run the replay twice
// per process on both streams against the oracle.
struct DevArena {
    char* p = nullptr;
    size_t cap = 0, used = 0;
    std::vector<char*> retired;
    ~DevArena() {
        if (p) (void)hipFree(p);
        for (char* r : retired) (void)hipFree(r);
    }
    static size_t round_up(size_t b) { return (std::max<size_t>(b, 1) + 255) & ~size_t(255); }
    // make room for `bytes` (the sum of round_up of every take of one replay)
    hipError_t reset(size_t bytes) {
        used = 0;
        if (bytes <= cap) return hipSuccess;
        if (p) retired.push_back(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 4, size_t(1) << 20);
        const double t = now_ms();
        const hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), want);
        g_devbuf_ns.fetch_add(int64_t((now_ms() - t) * 1e6));
        if (e == hipSuccess) cap = want;
        return e;
    }
    template <typename T>
    T* take(size_t count) {
        const size_t b = round_up(sizeof(T) * count);
        if (used + b > cap) return nullptr;
        T* r = reinterpret_cast<T*>(p + used);
        used += b;
        return r;
    }
};

// IntPower(10.0, -Precision) (encoder.lpr:761)
double scan_tolerance(int precision) {
    if (precision <= 0) return 1.0;
    double p = 1.0, base = 10.0;
    int i = precision;
    while (i > 0) {
        while ((i & 1) == 0) {
            i >>= 1;
            base = base * base;
        }
        --i;
        p = p * base;
    }
    return 1.0 / p;
}

// leaves of the batched kernel's layout: K rounded up to a power of two, at
// least 256 (a K below it runs the padded layout, gsc_tree.h pad_tree)
int padded_k(int K) {
    int k = 256;
    while (k < K) k <<= 1;
    return k;
}

// D in {8, 16, 32} and 2 <= K <= 4096: the batched speculative kernel
// (gsc_scan.hip) covers the pass (D = 32 with 2048 < K <= 4096 on one CU per
// frame in the split layout: the cepstrum half of each centroid in HBM).
bool batched_scan_shape(int D, int K) {
    if (std::getenv("GSC_SCAN_GENERIC")) return false;  // diagnostic switch
    return (D == 8 || D == 16 || D == 32) && K >= 2 && K <= 4096;
}

// split-layout tail array offset of frame i (frames' slots of the largest size)
int64_t tail_offset(int i) { return int64_t(i) * 4096 * 16; }

// launch rounds of launch_scan_passes since the last reset (bench: launches
// of the dominant kernel)
std::atomic<int> g_scan_rounds{0};

// all KNNScanReduce passes of a batch; converged frames exit early, the
// generic launch after a batched one only runs the frames the batched kernel
// handed over (NaN centroids)
hipError_t launch_scan_passes(int D, ReduceFrame* dfr, int nf, int K, const float* X, float* C, int* is, float* fs,
                              const float* rate, int precision) {
    const double tol = scan_tolerance(precision);
    const bool batched = batched_scan_shape(D, K);
    int logk = 0;
    while ((1 << logk) < padded_k(K)) ++logk;
    DevBuf<float> tails;  // split layout: every frame's tail features (ReduceFrame::t_off)
    if (batched && gsc_scan_tail_floats_per_frame(D, logk) > 0) {
        const hipError_t e = tails.alloc(size_t(tail_offset(nf)));
        if (e != hipSuccess) return e;
    }
    int max_passes = kMaxScanIters;
    if (const char* e = std::getenv("GSC_SCAN_MAX_PASSES")) max_passes = std::max(1, std::min(kMaxScanIters, std::atoi(e)));
    // every launch advances each live frame by at least one pass (the batched
    // kernel runs a frame until it converges or meets a NaN pass, which the
    // generic launch then takes), so max_passes rounds always suffice
    std::vector<int32_t> flags(2 * static_cast<size_t>(nf));  // (done, generic) per frame
    static_assert(offsetof(ReduceFrame, generic) == offsetof(ReduceFrame, done) + sizeof(int32_t), "adjacent flags");
    for (int round = 0; round < max_passes; ++round) {
        if (batched) {
            // opts bit 0 (diagnostic GSC_SCAN_FULL_A1): full-dimension A1 bounds in every pass
            // bit 1 (GSC_SCAN_NO_PRUNE, experiment): no per-wave A1 pruning
            // bits 8..15 (GSC_SCAN_KB, experiment): queries per speculative batch (below the kernel's 32)
            const int opts = (std::getenv("GSC_SCAN_FULL_A1") ? 1 : 0) | (std::getenv("GSC_SCAN_NO_PRUNE") ? 2 : 0) |
                             ((std::getenv("GSC_SCAN_KB") ? (std::atoi(std::getenv("GSC_SCAN_KB")) & 255) : 0) << 8);
            hipError_t e =
                gsc_launch_scan_batch(D, logk, dfr, nf, X, C, is, rate, tol, max_passes, opts, tails.p, nullptr);
            if (e != hipSuccess) return e;
            // the generic kernel runs only when the batched one handed a frame
            // over (an empty launch of it still costs ~30 ms: 256 large-LDS
            // workgroups); stop once every frame is done
            e = hipMemcpy2D(flags.data(), 2 * sizeof(int32_t), &dfr[0].done, sizeof(ReduceFrame), 2 * sizeof(int32_t),
                            size_t(nf), hipMemcpyDeviceToHost);
            if (e != hipSuccess) return e;
            g_scan_rounds.fetch_add(1);
            bool any_generic = false, all_done = true;
            for (int i = 0; i < nf; ++i) {
                all_done = all_done && flags[2 * size_t(i)] != 0;
                any_generic = any_generic || flags[2 * size_t(i) + 1] != 0;
            }
            if (all_done) break;
            if (!any_generic) continue;
        }
        const hipError_t e = gsc_launch_scan_pass(D, dfr, nf, K, X, C, is, fs, rate, tol, max_passes, batched ? 1 : 0, nullptr);
        if (e != hipSuccess) return e;
        if (!batched) g_scan_rounds.fetch_add(1);  // the generic kernel runs one pass per round
    }
    return hipSuccess;
}

// rate = Single(1/sqrt(cnt)) for cnt in [0, n] (encoder.lpr:735)
std::vector<float> rate_table(int n) {
    std::vector<float> t(size_t(n) + 2);
    t[0] = 0.0f;
    for (int c = 1; c < int(t.size()); ++c) t[c] = float(1.0 / std::sqrt(double(c)));
    return t;
}

// ---- batched device stages --------------------------------------------------

// Reduce (yakmo seeding + KNNScanReduce) for a batch of frames; X/C host arrays
// are concatenated per frame (N_f*D and K*D floats).
// X: device slab, frame i's N_i x D features at dX + xoff[i]
// cl_host / notify (optional, device pointers of host-mapped memory): the
// batched kernel copies a frame's final clusters to cl_host + its n_off and
// then sets notify[i], so the host can post-process it during the scan tail
// D: the slab's row width (8, 16 or 32); dcol: the real colCount 2*ChunkSize
// (<= D, trailing features zero; 0 = D)
int run_reduce_batch_dev(int D, int K, int precision, const std::vector<int>& Ns, const std::vector<int64_t>& xoff,
                         const float* dX, std::vector<float>* C, std::vector<int>* clusters, std::vector<int>* iters,
                         std::vector<int>* slow, long long* restarts, double* yakmo_ms, double* scan_ms,
                         int* cl_host = nullptr, int* notify = nullptr, int dcol = 0) {
    // launches: one yakmo launch + kMaxScanIters scan launches per batch
    const int nf = int(Ns.size());
    if (nf == 0) return 0;
    if (D != 8 && D != 16 && D != 32) return fail("KNNScanReduce kernels support D = 8, 16 or 32 (ChunkSize 4, 8, 16)");
    std::vector<ReduceFrame> fr(static_cast<size_t>(nf));
    int64_t no = 0, maxN = 0;
    for (int i = 0; i < nf; ++i) {
        fr[i] = ReduceFrame{};
        fr[i].x_off = xoff[i];
        fr[i].c_off = int64_t(i) * K * D;
        fr[i].n_off = no;
        fr[i].k_off = 0;  // filled below
        fr[i].N = Ns[i];
        fr[i].K = K;
        fr[i].dcol = dcol;
        no += Ns[i];
        maxN = std::max<int64_t>(maxN, Ns[i]);
    }
    const int Kp = padded_k(K);  // per-position scratch covers the padded layout
    for (int i = 0; i < nf; ++i) {
        fr[i].k_off = no + int64_t(i) * K;
        fr[i].ka_off = no + int64_t(nf) * K + int64_t(i) * Kp;
        fr[i].t_off = tail_offset(i);
        if (cl_host && notify) {
            fr[i].cl_host = cl_host + fr[i].n_off;
            fr[i].notify = notify + i;
        }
    }
    DevBuf<float> dC, dF, dRate, dYSum;
    DevBuf<int> dI;
    DevBuf<uint32_t> dBits;
    DevBuf<ReduceFrame> dFr;
    HIP_TRY(dC.alloc(size_t(nf) * K * D));
    HIP_TRY(dF.alloc(size_t(no) * 4));
    HIP_TRY(dI.alloc(size_t(no) + size_t(nf) * (size_t(K) + size_t(Kp))));
    if (maxN > gsc_yakmo_max_lds_points()) {  // long frames: yakmo's bitmap and prefix summaries in HBM
        HIP_TRY(dBits.alloc(gsc_yakmo_big_words(no, nf)));
        HIP_TRY(dYSum.alloc(gsc_yakmo_big_floats(no, nf)));
    }
    HIP_TRY(dFr.alloc(size_t(nf)));
    const std::vector<float> rt = rate_table(int(maxN));
    HIP_TRY(dRate.alloc(rt.size()));
    HIP_TRY(hipMemcpy(dRate.p, rt.data(), sizeof(float) * rt.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dFr.p, fr.data(), sizeof(ReduceFrame) * size_t(nf), hipMemcpyHostToDevice));
    hipEvent_t e0, e1, e2;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventCreate(&e2));
    HIP_TRY(hipEventRecord(e0, nullptr));
    HIP_TRY(gsc_launch_yakmo(D, dFr.p, nf, dX, dC.p, dF.p, dI.p, dYSum.p, dBits.p, int(maxN), nullptr));
    HIP_TRY(hipEventRecord(e1, nullptr));
    HIP_TRY(launch_scan_passes(D, dFr.p, nf, K, dX, dC.p, dI.p, dF.p, dRate.p, precision));
    HIP_TRY(hipEventRecord(e2, nullptr));
    HIP_TRY(hipEventSynchronize(e2));
    float t1 = 0, t2 = 0;
    (void)hipEventElapsedTime(&t1, e0, e1);
    (void)hipEventElapsedTime(&t2, e1, e2);
    if (yakmo_ms) *yakmo_ms += t1;
    if (scan_ms) *scan_ms += t2;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipEventDestroy(e2);
    C->resize(size_t(nf) * K * D);
    clusters->resize(size_t(no));
    HIP_TRY(hipMemcpy(C->data(), dC.p, sizeof(float) * C->size(), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(clusters->data(), dI.p, sizeof(int) * size_t(no), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(fr.data(), dFr.p, sizeof(ReduceFrame) * size_t(nf), hipMemcpyDeviceToHost));
    if (std::getenv("GSC_HOST_TIMING")) {  // spread of the frames' finishing times (the scan tail)
        std::vector<uint64_t> t;
        for (int i = 0; i < nf; ++i)
            if (fr[i].t_done) t.push_back(fr[i].t_done);
        if (!t.empty()) {
            std::sort(t.begin(), t.end());
            const double last = double(t.back());
            auto at = [&](double q) { return (last - double(t[size_t(q * double(t.size() - 1))])) / 1e5; };
            std::fprintf(stderr, "scan tail: frames finished [ms before the last] min %.1f p10 %.1f p50 %.1f p90 %.1f\n",
                         at(0.0), at(0.1), at(0.5), at(0.9));
        }
    }
    if (std::getenv("GSC_FRAME_STATS")) {  // diagnostic: per-frame chain length and finishing time
        uint64_t t0 = ~0ull;
        for (int i = 0; i < nf; ++i)
            if (fr[i].t_done) t0 = std::min<uint64_t>(t0, fr[i].t_done);
        for (int i = 0; i < nf; ++i)
            std::fprintf(stderr, "frame %d: N %d passes %d slow %d restarts %d done +%.1f ms\n", i, fr[i].N, fr[i].iters,
                         fr[i].slow, fr[i].restarts, fr[i].t_done ? double(fr[i].t_done - t0) / 1e5 : -1.0);
    }
    if (std::getenv("GSC_HOST_TIMING") && nf > 0 && fr[0].ystamps[6] + fr[0].ystamps[1] + fr[0].ystamps[2] != 0) {
        // stamps builds: yakmo phase clocks, mean over frames (cycles per pick)
        double m[16] = {};
        for (int i = 0; i < nf; ++i)
            for (int k = 0; k < 16; ++k) m[k] += double(fr[i].ystamps[k]) / double(nf) / double(K);
        std::fprintf(stderr,
                     "yakmo stamps [clk/pick]: chain pick %.0f fast %.0f slow %.0f wait %.0f (fast calls %.1f"
                     " slow blocks %.1f) | dist pick+sdlo %.0f compute %.0f wait %.0f | negative deltas dropped"
                     " per pick: chain %.3g dist %.3g\n",
                     m[0], m[1], m[2], m[3], m[4], m[5], m[8], m[9], m[10], m[6], m[14]);
    }
    iters->resize(size_t(nf));
    slow->resize(size_t(nf));
    for (int i = 0; i < nf; ++i) {
        (*iters)[i] = fr[i].iters;
        (*slow)[i] = fr[i].slow;
        if (restarts) *restarts += fr[i].restarts;
        if (fr[i].loop_iters < 0) return fail("KNNScanReduce: batched pipeline made no progress (guard tripped)");
    }
    return 0;
}

// host X: frames concatenated (N_f * D floats each)
int run_reduce_batch(int D, int K, int precision, const std::vector<int>& Ns, const std::vector<float>& X,
                     std::vector<float>* C, std::vector<int>* clusters, std::vector<int>* iters, std::vector<int>* slow,
                     long long* restarts, double* yakmo_ms, double* scan_ms) {
    std::vector<int64_t> xoff(Ns.size());
    int64_t xo = 0;
    for (size_t i = 0; i < Ns.size(); ++i) {
        xoff[i] = xo;
        xo += int64_t(Ns[i]) * D;
    }
    DevBuf<float> dX;
    HIP_TRY(dX.alloc(size_t(xo)));
    HIP_TRY(hipMemcpy(dX.p, X.data(), sizeof(float) * size_t(xo), hipMemcpyHostToDevice));
    return run_reduce_batch_dev(D, K, precision, Ns, xoff, dX.p, C, clusters, iters, slow, restarts, yakmo_ms,
                                scan_ms);
}

// KNNFit queries whose tie set exceeds ANN's 64-NN bucket (the brute-force
// kernel marks them -1): for each affected frame, the 4R candidate rows in
// the reference order f = 4c + 2neg + rev (encoder.lpr:928-938), ANN's kd-tree
// over them (the DLL's sequential build), and ANN's priority search + the tie
// rule for every such query (gsc_ann.hip knnfit_ann_kernel).
int run_knnfit_overflow(int CS, const std::vector<FitFrame>& fr, const std::vector<int>& ov_frames,
                        const std::vector<float>& eps, const std::vector<float>& cand, const std::vector<float>& q,
                        std::vector<int>* best, hipStream_t st, DevArena* arena) {
    const int nt = int(ov_frames.size());
    const double t_begin = now_ms();
    std::vector<float> pts;
    std::vector<int64_t> pt_off(static_cast<size_t>(nt)), nd_off(static_cast<size_t>(nt));
    std::vector<int> caps(static_cast<size_t>(nt));
    int64_t nodes = 0;
    int max_n = 0;
    for (int t = 0; t < nt; ++t) {
        const FitFrame& f = fr[size_t(ov_frames[t])];
        const int n = 4 * f.R;
        pt_off[t] = int64_t(pts.size());
        pts.resize(pts.size() + size_t(n) * CS);
        float* o = pts.data() + pt_off[t];
        const float* c = cand.data() + f.cand_off;
        for (int r = 0; r < f.R; ++r) {
            const float* v = c + size_t(r) * CS;
            for (int j = 0; j < CS; ++j) {
                const float fw = v[j], rv = v[CS - 1 - j];
                // makeFloatSample of the negated int16: exact negation, but 0 stays +0
                o[(size_t(4 * r) + 0) * CS + j] = fw;
                o[(size_t(4 * r) + 1) * CS + j] = rv;
                o[(size_t(4 * r) + 2) * CS + j] = fw == 0.0f ? 0.0f : -fw;
                o[(size_t(4 * r) + 3) * CS + j] = rv == 0.0f ? 0.0f : -rv;
            }
        }
        int p2 = 1;
        while (p2 < n) p2 <<= 1;
        caps[t] = 2 * p2;
        nd_off[t] = nodes;
        nodes += caps[t];
        max_n = std::max(max_n, n);
    }
    // jobs: every query the brute-force kernel flagged
    std::vector<KnnOvJob> jobs;
    std::vector<int64_t> job_q;
    for (int t = 0; t < nt; ++t) {
        const FitFrame& f = fr[size_t(ov_frames[t])];
        for (int i = 0; i < f.N; ++i)
            if ((*best)[size_t(f.out_off + i)] == -1) {
                jobs.push_back(KnnOvJob{t, int(f.q_off + int64_t(i) * CS), int(f.out_off + i), eps[size_t(ov_frames[t])]});
            }
    }
    if (jobs.empty()) return 0;
    if (q.size() > size_t(INT32_MAX)) return fail("KNNFit overflow: query slab exceeds 2^31 floats");
    // the box queues (<= one push per split node each): bounded launches
    const int pq_cap = max_n + 2;
    const size_t per_job = size_t(pq_cap) * (sizeof(float) + sizeof(int4));
    const int chunk = int(std::max<size_t>(64, std::min<size_t>(jobs.size(), (size_t(2) << 30) / per_job)));
    // the caller's arena (no allocation on the replay's stream, nothing freed
    // before the owner is done); every sub-buffer poison-filled below
    const size_t npts = pts.size() / size_t(CS);
    const size_t R = DevArena::round_up(sizeof(float) * pts.size()) + 2 * DevArena::round_up(sizeof(float) * npts) +
                     2 * DevArena::round_up(sizeof(int) * size_t(nodes)) + 2 * DevArena::round_up(sizeof(float) * size_t(nodes)) +
                     DevArena::round_up(sizeof(int) * npts) + DevArena::round_up(sizeof(float) * size_t(2 * CS * nt)) +
                     DevArena::round_up(sizeof(AnnTree) * size_t(nt)) + DevArena::round_up(sizeof(float) * q.size()) +
                     DevArena::round_up(sizeof(int) * best->size()) + DevArena::round_up(sizeof(KnnOvJob) * jobs.size()) +
                     DevArena::round_up(sizeof(float) * size_t(chunk) * pq_cap) +
                     DevArena::round_up(sizeof(int4) * size_t(chunk) * pq_cap);
    HIP_TRY(arena->reset(R));
    float* dPts = arena->take<float>(pts.size());
    int* dPidx = arena->take<int>(npts);
    float* dVal = arena->take<float>(npts);
    int* dCd = arena->take<int>(size_t(nodes));
    float* dCv = arena->take<float>(size_t(nodes));
    float* dLo = arena->take<float>(size_t(nodes));
    float* dHi = arena->take<float>(size_t(nodes));
    float* dBnd = arena->take<float>(size_t(2 * CS * nt));
    AnnTree* dTrees = arena->take<AnnTree>(size_t(nt));
    float* dQ = arena->take<float>(q.size());
    int* dOut = arena->take<int>(best->size());
    KnnOvJob* dJobs = arena->take<KnnOvJob>(jobs.size());
    float* dPqk = arena->take<float>(size_t(chunk) * pq_cap);
    int4* dPqn = arena->take<int4>(size_t(chunk) * pq_cap);
    (void)dVal;
    if (!dPqn) return fail("KNNFit overflow: replay arena too small");
    HIP_TRY(hipMemsetAsync(arena->p, 0xff, arena->used, st));  // poison (dCd's -1 marks unbuilt nodes too)
    HIP_TRY(hipMemcpyAsync(dPts, pts.data(), sizeof(float) * pts.size(), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(dQ, q.data(), sizeof(float) * q.size(), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(dOut, best->data(), sizeof(int) * best->size(), hipMemcpyHostToDevice, st));
    std::vector<AnnTree> trees(static_cast<size_t>(nt));
    for (int t = 0; t < nt; ++t) {
        AnnTree& a = trees[size_t(t)];
        a.pts = dPts + pt_off[t];
        a.n = 4 * fr[size_t(ov_frames[t])].R;
        a.dd = CS;
        a.pidx = dPidx + pt_off[t] / CS;
        a.cd = dCd + nd_off[t];
        a.cv = dCv + nd_off[t];
        a.lo = dLo + nd_off[t];
        a.hi = dHi + nd_off[t];
        a.bnd = dBnd + size_t(2 * CS) * size_t(t);
        a.val = dVal + pt_off[t] / CS;
        a.ncap = caps[t];
    }
    HIP_TRY(hipMemcpyAsync(dTrees, trees.data(), sizeof(AnnTree) * size_t(nt), hipMemcpyHostToDevice, st));
    const bool timing = std::getenv("GSC_HOST_TIMING") != nullptr;
    struct EvPair {  // diagnostic events, released on every return path
        hipEvent_t a = nullptr, b = nullptr;
        ~EvPair() {
            if (a) (void)hipEventDestroy(a);
            if (b) (void)hipEventDestroy(b);
        }
    } ev;
    hipEvent_t& eb0 = ev.a;
    hipEvent_t& eb1 = ev.b;
    if (timing) {
        HIP_TRY(hipEventCreate(&eb0));
        HIP_TRY(hipEventCreate(&eb1));
        HIP_TRY(hipEventRecord(eb0, st));
    }
    HIP_TRY(gsc_launch_ann_build_many(dTrees, nt, st));
    if (timing) HIP_TRY(hipEventRecord(eb1, st));
    HIP_TRY(hipMemcpyAsync(dJobs, jobs.data(), sizeof(KnnOvJob) * jobs.size(), hipMemcpyHostToDevice, st));
    for (size_t j0 = 0; j0 < jobs.size(); j0 += size_t(chunk)) {
        const int nj = int(std::min<size_t>(size_t(chunk), jobs.size() - j0));
        HIP_TRY(gsc_launch_knnfit_ann(dTrees, dJobs + j0, nj, dQ, dOut, dPqk, dPqn, pq_cap, st));
    }
    HIP_TRY(hipMemcpyAsync(best->data(), dOut, sizeof(int) * best->size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (timing) {
        float bms = 0.0f;
        (void)hipEventElapsedTime(&bms, eb0, eb1);
        std::fprintf(stderr, "KNNFit overflow: %d trees (largest %d candidates), %zu queries, %.2f ms (tree builds %.2f ms)\n",
                     nt, max_n, jobs.size(), now_ms() - t_begin, double(bms));
    }
    for (const KnnOvJob& j : jobs) {
        const int b = (*best)[size_t(j.out)];
        if (b == -4) return fail("KNNFit overflow: a tree index left its frame's arrays (device bounds check)");
        if (b < 0) return fail("KNNFit: ANN priority search emulation failed");
    }
    return 0;
}

// q: host queries, or empty with qdev = the device query slab (same layout)
int run_knnfit_batch(int CS, const std::vector<int>& Rs, const std::vector<int>& Ns, const std::vector<float>& eps,
                     const std::vector<float>& cand, const std::vector<float>& q, std::vector<int>* best,
                     double* knn_ms, const float* qdev = nullptr) {
    const int nf = int(Ns.size());
    if (nf == 0) return 0;
    std::vector<FitFrame> fr(static_cast<size_t>(nf));
    int64_t co = 0, qo = 0;
    int maxN = 0, maxR = 0;
    for (int i = 0; i < nf; ++i) {
        fr[i] = FitFrame{};
        fr[i].cand_off = co;
        fr[i].q_off = qo;
        fr[i].out_off = qo / CS;
        fr[i].R = Rs[i];
        fr[i].N = Ns[i];
        fr[i].eps = eps[i];
        co += int64_t(Rs[i]) * CS;
        qo += int64_t(Ns[i]) * CS;
        maxN = std::max(maxN, Ns[i]);
        maxR = std::max(maxR, Rs[i]);
    }
    DevBuf<float> dCand, dQ;
    DevBuf<int> dOut;
    DevBuf<FitFrame> dFr;
    HIP_TRY(dCand.alloc(size_t(co)));
    if (!qdev) {
        HIP_TRY(dQ.alloc(size_t(qo)));
        HIP_TRY(hipMemcpy(dQ.p, q.data(), sizeof(float) * size_t(qo), hipMemcpyHostToDevice));
        qdev = dQ.p;
    }
    HIP_TRY(dOut.alloc(size_t(qo / CS)));
    HIP_TRY(dFr.alloc(size_t(nf)));
    HIP_TRY(hipMemcpy(dCand.p, cand.data(), sizeof(float) * size_t(co), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dFr.p, fr.data(), sizeof(FitFrame) * size_t(nf), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, nullptr));
    HIP_TRY(gsc_launch_knnfit(CS, dFr.p, nf, maxN, maxR, dCand.p, qdev, dOut.p, nullptr));
    HIP_TRY(hipEventRecord(e1, nullptr));
    HIP_TRY(hipEventSynchronize(e1));
    float t = 0;
    (void)hipEventElapsedTime(&t, e0, e1);
    if (knn_ms) *knn_ms += t;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    best->resize(size_t(qo / CS));
    HIP_TRY(hipMemcpy(best->data(), dOut.p, sizeof(int) * best->size(), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(fr.data(), dFr.p, sizeof(FitFrame) * size_t(nf), hipMemcpyDeviceToHost));
    std::vector<int> ov_frames;
    for (int i = 0; i < nf; ++i)
        if (fr[i].overflow > 0) ov_frames.push_back(i);
    if (!ov_frames.empty()) {
        const double t0 = now_ms();
        std::vector<float> qh;
        if (q.empty()) {  // the overflow replay reads host queries
            qh.resize(size_t(qo));
            HIP_TRY(hipMemcpy(qh.data(), qdev, sizeof(float) * size_t(qo), hipMemcpyDeviceToHost));
        }
        DevArena arena;  // synchronous call: freed on return, after the stream sync
        if (run_knnfit_overflow(CS, fr, ov_frames, eps, cand, q.empty() ? qh : q, best, nullptr, &arena) != 0) return -1;
        if (knn_ms) *knn_ms += now_ms() - t0;
    }
    return 0;
}

// Pinned host staging, kept across encode calls (pinning ~100 MB per call
// would cost more than the transfers).  Leaked on purpose: it lives until the
// process exits, after the HIP runtime may already be gone.
struct PinnedBuf {
    unsigned flags = hipHostMallocDefault;
    void* p = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
        const hipError_t e = hipHostMalloc(&p, want, flags);
        if (e == hipSuccess) cap = want;
        return e;
    }
    template <typename T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

struct PinnedArena {
    std::mutex m;
    // host-side DMA staging: candidates up, use counts down, remap up, words down, codes down
    PinnedBuf cand, cnt, remap, words, codes;
    // written by the scan kernel (fine-grained, mapped): final clusters and done flags
    PinnedBuf cl{hipHostMallocMapped | hipHostMallocCoherent}, notify{hipHostMallocMapped | hipHostMallocCoherent};
};

PinnedArena& pinned_arena() {
    static PinnedArena* a = new PinnedArena;
    return *a;
}

}  // namespace

// KNNFit + prune/sort + index packing of one encode, run on frame groups as
// they become ready (frames that skip the Reduce at once, reduced frames when
// the scan kernel signals them), on its own non-blocking stream so that the
// groups run on the CUs that finished frames leave idle.
struct PostCtx {
    hipStream_t st = nullptr;
    bool recon = false;
    std::vector<int64_t> coff, roff, woff, noff;  // per frame: candidates (floats), R slots, words, chunks
    DevBuf<float> dCand;
    DevBuf<int> dBest, dCnt, dRemap;
    DevBuf<uint32_t> dWords, dCodes;
    DevBuf<FitFrame> dFit;
    DevBuf<PackFrame> dPack;
    DevArena ov_arena;  // KNNFit overflow replay scratch (kept until the encode is done)
    const float* dQry = nullptr;
    float* hCand = nullptr;
    int *hCnt = nullptr, *hRemap = nullptr;
    uint32_t *hWords = nullptr, *hCodes = nullptr;
    int slot = 0;  // next descriptor slot in dFit / dPack
    double knn_ms = 0;
    int groups = 0;
    long long ov_queries = 0;  // KNNFit queries replayed through ANN's priority search
    ~PostCtx() {
        if (st) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
    }
};

// rows of `dp` floats (the device slab) -> rows of the first `d` of them
static void compact_rows(std::vector<float>* v, int n, int dp, int d) {
    if (dp == d) return;
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < d; ++k) (*v)[size_t(i) * d + k] = (*v)[size_t(i) * dp + k];
    v->resize(size_t(n) * d);
}

// ---- Encoder::device_dsp: FindAttenuationDivider + features on the device --
// dXv: DevBuf<float>* that receives the feature slab (kept for the Reduce).
int Encoder::device_dsp(int b, std::vector<FrameState>& frames, void* dXv, std::vector<int64_t>* xoff, double* ms,
                        std::string* err, void* dQv) {
    auto& dX = *static_cast<DevBuf<float>*>(dXv);
    const int cs = opt_.chunk_size, ch = channels_, nfr = int(frames.size());
    const int obd = (1 << (opt_.chunk_bit_depth - 1)) - 1;
    const int e = b + nfr;
    const int64_t s_first = fr_start_[b], span = int64_t(fr_end_[e - 1]) - s_first + 1;
    std::vector<DspFrame> df(static_cast<size_t>(nfr));
    xoff->assign(size_t(nfr), 0);
    int64_t xo = 0, co = 0;
    int max_n = 0;
    for (int i = 0; i < nfr; ++i) {
        const FrameState& f = frames[i];
        df[i] = DspFrame{};
        df[i].s_off = int64_t(f.start) - s_first;
        df[i].x_off = xo;
        df[i].c_off = co;
        df[i].sc = f.sample_count;
        df[i].n = f.n;
        (*xoff)[i] = xo;
        xo += int64_t(f.n) * feature_stride(cs);
        co += f.n;
        max_n = std::max(max_n, f.n);
    }
    std::vector<double> trig;
    double s0 = 0, scale = 0;
    trig_pack(cs, &trig, &s0, &scale);
    DevBuf<double> dS, dT;
    DevBuf<DspFrame> dF;
    DevBuf<uint8_t> dNR;
    DevBuf<int16_t> dP;
    float* dQ = nullptr;
    const double t0 = now_ms();
    if (dS.alloc(size_t(ch) * size_t(span)) != hipSuccess || dT.alloc(trig.size()) != hipSuccess ||
        dF.alloc(size_t(nfr)) != hipSuccess || dNR.alloc(size_t(co)) != hipSuccess || dX.alloc(size_t(xo)) != hipSuccess ||
        dP.alloc(size_t(ch) * size_t(span)) != hipSuccess) {
        *err = "device DSP: out of device memory";
        return -1;
    }
    if (dQv) {
        auto& q = *static_cast<DevBuf<float>*>(dQv);
        if (q.alloc(size_t(co) * size_t(cs)) != hipSuccess) {
            *err = "device DSP: out of device memory";
            return -1;
        }
        dQ = q.p;
    }
    auto chk = [&](hipError_t r, const char* what) {
        if (r == hipSuccess) return true;
        *err = std::string("device DSP: ") + what + ": " + hipGetErrorString(r);
        return false;
    };
    // the SmallInt samples of the span (a quarter of the f64 bytes), converted on the device
    if (!chk(hipMemcpy(dP.p, pcm_.data() + size_t(s_first - pcm_off_) * ch, sizeof(int16_t) * size_t(ch) * size_t(span),
                       hipMemcpyHostToDevice),
             "sample upload") ||
        !chk(gsc_launch_pcm(dP.p, span, ch, dS.p, nullptr), "sample conversion"))
        return -1;
    if (!chk(hipMemcpy(dT.p, trig.data(), sizeof(double) * trig.size(), hipMemcpyHostToDevice), "trig upload") ||
        !chk(hipMemcpy(dF.p, df.data(), sizeof(DspFrame) * size_t(nfr), hipMemcpyHostToDevice), "frame upload") ||
        !chk(gsc_launch_atten(cs, dF.p, nfr, dS.p, span, ch, obd, nullptr), "atten launch") ||
        !chk(gsc_launch_features(cs, dF.p, nfr, max_n, dS.p, span, ch, dT.p, s0, scale, dX.p, dNR.p, dQ, nullptr),
             "features launch"))
        return -1;
    std::vector<uint8_t> nr(static_cast<size_t>(co));
    if (!chk(hipMemcpy(df.data(), dF.p, sizeof(DspFrame) * size_t(nfr), hipMemcpyDeviceToHost), "frame download") ||
        !chk(hipMemcpy(nr.data(), dNR.p, size_t(co), hipMemcpyDeviceToHost), "flag download"))
        return -1;
    for (int i = 0; i < nfr; ++i) {
        FrameState& f = frames[i];
        f.atten_div = df[i].atten_div;
        const uint8_t* q = nr.data() + df[i].c_off;
        for (int c = 0; c < f.n; ++c) {
            f.neg[c] = q[c] & 1;
            f.rev[c] = (q[c] >> 1) & 1;
        }
    }
    if (ms) *ms += now_ms() - t0;
    return 0;
}

// ---- Encoder::device_recon: reconstruction + PsyADelta numerator (f4) -----
int Encoder::device_recon(int b, const std::vector<FrameState>& frames, ReconOut* ro, std::string* err) {
    const int cs = opt_.chunk_size, ch = channels_, nfr = int(frames.size());
    if (nfr == 0) return 0;
    const double t0 = now_ms();
    const int64_t s_first = fr_start_[b], span = int64_t(fr_end_[b + nfr - 1]) - s_first + 1;
    std::vector<ReconFrame> rf(static_cast<size_t>(nfr));
    int64_t nchunk = 0, nred = 0;
    int max_n = 0;
    for (int i = 0; i < nfr; ++i) {
        const FrameState& f = frames[i];
        rf[i] = ReconFrame{nchunk, nred, int64_t(f.start) - s_first, f.n, f.sample_count, 1.0 / double(f.atten_div)};
        nchunk += f.n;
        nred += f.r;
        max_n = std::max(max_n, f.n);
    }
    std::vector<uint32_t> words(static_cast<size_t>(nchunk));
    std::vector<int16_t> rdst(static_cast<size_t>(std::max<int64_t>(nred, 1) * cs));
    std::vector<uint8_t> ratten(static_cast<size_t>(std::max<int64_t>(nred, 1)));
    parallel_for(nfr, host_threads(), [&](int i) {
        const FrameState& f = frames[i];
        uint32_t* w = words.data() + rf[i].chunk_off;
        for (int c = 0; c < f.n; ++c) w[c] = uint32_t(f.red[c]) << 2 | uint32_t(f.neg[c] & 1) << 1 | uint32_t(f.rev[c] & 1);
        std::copy(f.rdst.begin(), f.rdst.begin() + long(size_t(f.r) * cs), rdst.begin() + long(rf[i].red_off * cs));
        std::copy(f.ratten.begin(), f.ratten.begin() + f.r, ratten.begin() + long(rf[i].red_off));
    });
    // srcData of the range (SmallInt, zero past the file's own samples: PrepareFrames pads, encoder.lpr:1317-1323)
    const int64_t psc = ro->wav_len >= 44 ? int64_t((ro->wav_len - 44) / (2 * size_t(ch))) : 0;
    std::vector<int16_t> src(static_cast<size_t>(span * ch), 0);
    const int64_t avail = std::max<int64_t>(0, std::min(span, psc - s_first));
    if (avail > 0) std::memcpy(src.data(), ro->wav + 44 + size_t(s_first) * ch * 2, size_t(avail) * ch * 2);
    DevBuf<ReconFrame> dF;
    DevBuf<uint32_t> dW;
    DevBuf<int16_t> dR, dOut, dSrc;
    DevBuf<uint8_t> dA;
    DevBuf<unsigned long long> dAcc;
    auto chk = [&](hipError_t r, const char* what) {
        if (r == hipSuccess) return true;
        *err = std::string("reconstruction: ") + what + ": " + hipGetErrorString(r);
        return false;
    };
    const size_t nout = size_t(span) * ch;
    if (!chk(dF.alloc(size_t(nfr)), "alloc") || !chk(dW.alloc(words.size()), "alloc") ||
        !chk(dR.alloc(rdst.size()), "alloc") || !chk(dA.alloc(ratten.size()), "alloc") ||
        !chk(dOut.alloc(nout), "alloc") || !chk(dSrc.alloc(nout), "alloc") || !chk(dAcc.alloc(1), "alloc"))
        return -1;
    if (!chk(hipMemcpy(dF.p, rf.data(), sizeof(ReconFrame) * rf.size(), hipMemcpyHostToDevice), "upload") ||
        !chk(hipMemcpy(dW.p, words.data(), sizeof(uint32_t) * words.size(), hipMemcpyHostToDevice), "upload") ||
        !chk(hipMemcpy(dR.p, rdst.data(), sizeof(int16_t) * rdst.size(), hipMemcpyHostToDevice), "upload") ||
        !chk(hipMemcpy(dA.p, ratten.data(), ratten.size(), hipMemcpyHostToDevice), "upload") ||
        !chk(hipMemcpy(dSrc.p, src.data(), sizeof(int16_t) * nout, hipMemcpyHostToDevice), "upload") ||
        !chk(hipMemset(dOut.p, 0, sizeof(int16_t) * nout), "memset") ||  // dstData starts zeroed (encoder.lpr:497-501)
        !chk(hipMemset(dAcc.p, 0, sizeof(unsigned long long)), "memset") ||
        !chk(gsc_launch_recon(dF.p, nfr, max_n, cs, ch, opt_.chunk_bit_depth, dW.p, dR.p, dA.p, dOut.p, nullptr),
             "recon launch") ||
        !chk(gsc_launch_sqdiff(dSrc.p, dOut.p, int64_t(nout), dAcc.p, nullptr), "PsyADelta launch"))
        return -1;
    unsigned long long sq = 0;
    if (!chk(hipMemcpy(ro->pcm + size_t(s_first) * ch, dOut.p, sizeof(int16_t) * nout, hipMemcpyDeviceToHost),
             "download") ||
        !chk(hipMemcpy(&sq, dAcc.p, sizeof(sq), hipMemcpyDeviceToHost), "download"))
        return -1;
    ro->sq += sq;
    ro->ms += now_ms() - t0;
    return 0;
}

// test hook (tests/test_gpu_encoder.py): GSC_TEST_FAIL_POST set makes ONE
// post_group call of the process fail, while the scan may still be running
static bool inject_post_failure() {
    static std::atomic<int> used{0};
    return std::getenv("GSC_TEST_FAIL_POST") != nullptr && used.exchange(1) == 0;
}

int Encoder::post_group(std::vector<FrameState>& frames, const std::vector<int>& ids,
                        const std::vector<char>& reduced, PostCtx& c, std::string* err) {
    const int cs = opt_.chunk_size, bd = opt_.chunk_bit_depth, obd = (1 << (bd - 1)) - 1;
    const int g = int(ids.size());
    if (g == 0) return 0;
    if (inject_post_failure()) {
        *err = "injected post_group failure (GSC_TEST_FAIL_POST)";
        return -1;
    }
    auto chk = [&](hipError_t r, const char* what) {
        if (r == hipSuccess) return true;
        *err = std::string("KNNFit/pack pipeline: ") + what + ": " + hipGetErrorString(r);
        return false;
    };
    std::vector<float> eps(static_cast<size_t>(g));
    // TFrame.Reduce's tail (cluster means, sort, reduced chunks) and the
    // KNNFit candidates (encoder.lpr:843-889, 928-938), per frame on the host pool
    parallel_for(g, host_threads(), [&](int k) {
        FrameState& f = frames[size_t(ids[k])];
        frame_reduce_post(f, reduced[size_t(ids[k])] != 0);
        const double law = 1.0 / double(f.atten_div);
        // epsilon (encoder.lpr:940-943), accumulated in Single
        float acc = 1.0f;
        for (int j = 0; j <= 15; ++j) acc = float(double(acc) + double(j) * law);
        const float e1 = 1.0f / (float(1 << bd) * acc);
        const float e2 = float(1.0 / 32767.0);
        eps[size_t(k)] = e1 > e2 ? e1 : e2;
        float* cp = c.hCand + c.coff[size_t(ids[k])];
        for (int r = 0; r < f.r; ++r) {
            double coeff = 1.0;
            for (int a = 0; a <= f.ratten[r]; ++a) coeff += double(a) * law;
            for (int j = 0; j < cs; ++j) {
                double v = double(f.rdst[size_t(r) * cs + j]) / (double(obd) * coeff);
                v = std::min(1.0, std::max(-1.0, v));
                *cp++ = float(v);
            }
        }
    });
    const int gb = c.slot;
    c.slot += g;
    std::vector<FitFrame> fit(static_cast<size_t>(g));
    std::vector<PackFrame> pk(static_cast<size_t>(g));
    int maxN = 0, maxR = 0;
    for (int k = 0; k < g; ++k) {
        const size_t i = size_t(ids[k]);
        const FrameState& f = frames[i];
        fit[size_t(k)] = FitFrame{c.coff[i], c.noff[i] * cs, c.noff[i], f.r, f.n, eps[size_t(k)], 0};
        pk[size_t(k)] = PackFrame{c.noff[i], c.roff[i], c.woff[i], f.n, f.r, 0, 0};
        maxN = std::max(maxN, f.n);
        maxR = std::max(maxR, f.r);
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (!chk(hipEventCreate(&e0), "event") || !chk(hipEventCreate(&e1), "event")) return -1;
    struct EvGuard {
        hipEvent_t a, b;
        ~EvGuard() {
            (void)hipEventDestroy(a);
            (void)hipEventDestroy(b);
        }
    } evg{e0, e1};
    const hipStream_t st = c.st;
    bool ok = chk(hipMemcpyAsync(c.dFit.p + gb, fit.data(), sizeof(FitFrame) * size_t(g), hipMemcpyHostToDevice, st),
                  "upload") &&
              chk(hipMemcpyAsync(c.dPack.p + gb, pk.data(), sizeof(PackFrame) * size_t(g), hipMemcpyHostToDevice, st),
                  "upload");
    for (int k = 0; ok && k < g; ++k) {
        const size_t i = size_t(ids[k]);
        ok = chk(hipMemcpyAsync(c.dCand.p + c.coff[i], c.hCand + c.coff[i], sizeof(float) * size_t(frames[i].r) * cs,
                                hipMemcpyHostToDevice, st),
                 "candidate upload");
    }
    ok = ok && chk(hipEventRecord(e0, st), "event") &&
         chk(gsc_launch_knnfit(cs, c.dFit.p + gb, g, maxN, maxR, c.dCand.p, c.dQry, c.dBest.p, st), "KNNFit launch") &&
         chk(hipEventRecord(e1, st), "event") &&
         chk(gsc_launch_usecount(c.dPack.p + gb, g, c.dBest.p, c.dCnt.p, st), "use count launch") &&
         chk(hipMemcpyAsync(fit.data(), c.dFit.p + gb, sizeof(FitFrame) * size_t(g), hipMemcpyDeviceToHost, st),
             "download");
    for (int k = 0; ok && k < g; ++k) {
        const size_t i = size_t(ids[k]);
        ok = chk(hipMemcpyAsync(c.hCnt + c.roff[i], c.dCnt.p + c.roff[i], sizeof(int) * size_t(frames[i].r),
                                hipMemcpyDeviceToHost, st),
                 "use count download");
    }
    if (!ok || !chk(hipStreamSynchronize(st), "KNNFit")) return -1;
    float t = 0;
    if (hipEventElapsedTime(&t, e0, e1) == hipSuccess) c.knn_ms += t;
    // queries whose tie set exceeds ANN's 64-NN bucket: ANN's priority search
    // over the frame's candidate tree (rare; it waits for the scan)
    std::vector<int> ovk;
    for (int k = 0; k < g; ++k)
        if (fit[size_t(k)].overflow > 0) ovk.push_back(k);
    if (!ovk.empty()) {
        const double t0 = now_ms();
        std::vector<FitFrame> lf;
        std::vector<float> lcand, lq, leps;
        std::vector<int> lbest, lidx;
        for (int k : ovk) {
            const FrameState& f = frames[size_t(ids[k])];
            FitFrame x = fit[size_t(k)];
            x.cand_off = int64_t(lcand.size());
            x.q_off = int64_t(lq.size());
            x.out_off = int64_t(lbest.size());
            lcand.insert(lcand.end(), c.hCand + fit[size_t(k)].cand_off,
                         c.hCand + fit[size_t(k)].cand_off + size_t(f.r) * cs);
            lq.resize(lq.size() + size_t(f.n) * cs);
            lbest.resize(lbest.size() + size_t(f.n));
            if (!chk(hipMemcpyAsync(lq.data() + x.q_off, c.dQry + fit[size_t(k)].q_off, sizeof(float) * size_t(f.n) * cs,
                                    hipMemcpyDeviceToHost, st),
                     "query download") ||
                !chk(hipMemcpyAsync(lbest.data() + x.out_off, c.dBest.p + fit[size_t(k)].out_off,
                                    sizeof(int) * size_t(f.n), hipMemcpyDeviceToHost, st),
                     "download"))
                return -1;
            lidx.push_back(int(lf.size()));
            leps.push_back(x.eps);
            lf.push_back(x);
        }
        if (!chk(hipStreamSynchronize(st), "download")) return -1;
        c.ov_queries += std::count(lbest.begin(), lbest.end(), -1);
        if (run_knnfit_overflow(cs, lf, lidx, leps, lcand, lq, &lbest, st, &c.ov_arena) != 0) {
            *err = t_err;
            return -1;
        }
        for (size_t j = 0; j < ovk.size(); ++j)
            if (!chk(hipMemcpyAsync(c.dBest.p + fit[size_t(ovk[j])].out_off, lbest.data() + lf[j].out_off,
                                    sizeof(int) * size_t(lf[j].N), hipMemcpyHostToDevice, st),
                     "upload"))
                return -1;
        ok = chk(gsc_launch_usecount(c.dPack.p + gb, g, c.dBest.p, c.dCnt.p, st), "use count launch");
        for (int k = 0; ok && k < g; ++k) {
            const size_t i = size_t(ids[k]);
            ok = chk(hipMemcpyAsync(c.hCnt + c.roff[i], c.dCnt.p + c.roff[i], sizeof(int) * size_t(frames[i].r),
                                    hipMemcpyDeviceToHost, st),
                     "use count download");
        }
        if (!ok || !chk(hipStreamSynchronize(st), "use counts")) return -1;
        c.knn_ms += now_ms() - t0;
    }
    // prune + sort by use count on the host, then the index stream on the device
    parallel_for(g, host_threads(), [&](int k) {
        const size_t i = size_t(ids[k]);
        frame_prune(frames[i], c.hCnt + c.roff[i], c.hRemap + c.roff[i]);
    });
    // SaveStream's Assert(reducedChunks.Count <= CMaxChunksPerFrame) (encoder.lpr:986;
    // built with assertions on): only a -pr0 passthrough frame (KNNFit over
    // every chunk) can keep more than 4096 entries after pruning
    for (int k = 0; k < g; ++k) {
        const FrameState& f = frames[size_t(ids[k])];
        if (f.r > kMaxK) {
            *err = "SaveStream: Assert(reducedChunks.Count <= CMaxChunksPerFrame) failed: frame " +
                   std::to_string(f.index) + " keeps " + std::to_string(f.r) + " reduced chunks";
            return -1;
        }
    }
    ok = true;
    for (int k = 0; ok && k < g; ++k) {
        const size_t i = size_t(ids[k]);
        ok = chk(hipMemcpyAsync(c.dRemap.p + c.roff[i], c.hRemap + c.roff[i],
                                sizeof(int) * size_t(frames[i].r_before_prune), hipMemcpyHostToDevice, st),
                 "remap upload");
    }
    ok = ok && chk(gsc_launch_pack(c.dPack.p + gb, g, c.dBest.p, c.dRemap.p, c.dWords.p, c.recon ? c.dCodes.p : nullptr,
                                   st),
                   "pack launch") &&
         chk(hipMemcpyAsync(pk.data(), c.dPack.p + gb, sizeof(PackFrame) * size_t(g), hipMemcpyDeviceToHost, st),
             "download") &&
         chk(hipStreamSynchronize(st), "pack");
    for (int k = 0; ok && k < g; ++k) {
        const size_t i = size_t(ids[k]);
        const int64_t nw = (int64_t(pk[size_t(k)].nbits) + 31) / 32;  // whole u32 words (>= the 16-bit words used)
        if (pk[size_t(k)].nbits < 0 || nw > pack_word_capacity(frames[i].n)) {  // pack_kernel refused the overrun
            *err = "index packer overran its word slab";
            return -1;
        }
        ok = chk(hipMemcpyAsync(c.hWords + c.woff[i], c.dWords.p + c.woff[i], sizeof(uint32_t) * size_t(nw),
                                hipMemcpyDeviceToHost, st),
                 "stream download");
        if (ok && c.recon)
            ok = chk(hipMemcpyAsync(c.hCodes + c.noff[i], c.dCodes.p + c.noff[i], sizeof(uint32_t) * size_t(frames[i].n),
                                    hipMemcpyDeviceToHost, st),
                     "code download");
    }
    if (!ok || !chk(hipStreamSynchronize(st), "stream download")) return -1;
    parallel_for(g, host_threads(), [&](int k) {
        const size_t i = size_t(ids[k]);
        FrameState& f = frames[i];
        frame_save_head(f);
        const size_t nbytes = size_t((pk[size_t(k)].nbits + 15) / 16) * 2;  // 16-bit words, the last zero-padded
        const uint8_t* wb = reinterpret_cast<const uint8_t*>(c.hWords + c.woff[i]);
        f.stream.insert(f.stream.end(), wb, wb + nbytes);
        if (c.recon) {  // final index / dstNegative / dstReversed per chunk (reconstruction)
            f.red.resize(size_t(f.n));
            f.neg.resize(size_t(f.n));
            f.rev.resize(size_t(f.n));
            const uint32_t* cw = c.hCodes + c.noff[i];
            for (int j = 0; j < f.n; ++j) {
                f.red[size_t(j)] = int(cw[j] >> 2);
                f.neg[size_t(j)] = uint8_t((cw[j] >> 1) & 1);
                f.rev[size_t(j)] = uint8_t(cw[j] & 1);
            }
        }
    });
    c.groups += 1;
    return 0;
}

int Encoder::dsp_frame(int fi, int* atten_div, std::vector<float>* feat, std::string* err) {
    if (ensure_device() != 0) {
        *err = t_err;
        return -1;
    }
    if (fi < 0 || fi >= frame_count()) {
        *err = "frame index out of range";
        return -1;
    }
    warm_trig_tables(opt_.chunk_size);
    std::vector<FrameState> frames(1);
    frames[0].index = fi;
    frames[0].start = fr_start_[fi];
    frames[0].sample_count = fr_end_[fi] - fr_start_[fi] + 1;
    frame_host_src(frames[0]);
    DevBuf<float> dX;
    std::vector<int64_t> xoff;
    if (device_dsp(fi, frames, &dX, &xoff, nullptr, err) != 0) return -1;
    *atten_div = frames[0].atten_div;
    const int dp = feature_stride(opt_.chunk_size);
    feat->resize(size_t(frames[0].n) * dp);
    if (hipMemcpy(feat->data(), dX.p, sizeof(float) * feat->size(), hipMemcpyDeviceToHost) != hipSuccess) {
        *err = "feature download failed";
        return -1;
    }
    compact_rows(feat, frames[0].n, dp, 2 * opt_.chunk_size);
    return 0;
}

// ---- Encoder::encode_range: host srcData, device DSP + hot path ------------
int Encoder::encode_range(int b, int e, std::vector<uint8_t>* out, std::string* err, gsc_timing* tim,
                          ReconOut* recon, std::vector<size_t>* frame_bytes) {
    if (ensure_device() != 0) {
        *err = t_err;
        return -1;
    }
    const int cs = opt_.chunk_size, D = 2 * cs, K = opt_.chunks_per_frame;
    const int DP = feature_stride(cs);  // the feature slab's row width (D features, then zeros)
    const int nfr = e - b;
    std::vector<FrameState> frames(static_cast<size_t>(std::max(nfr, 0)));
    double t0 = now_ms();
    warm_trig_tables(cs);  // FPC trig tables, built before the workers start
    parallel_for(nfr, host_threads(), [&](int i) {
        FrameState& f = frames[i];
        f.index = b + i;
        f.start = fr_start_[b + i];
        f.sample_count = fr_end_[b + i] - fr_start_[b + i] + 1;
        frame_host_src(f);
    });
    double dsp_ms = 0;
    DevBuf<float> dFeat, dQry;
    std::vector<int64_t> feat_off;
    if (nfr > 0 && device_dsp(b, frames, &dFeat, &feat_off, &dsp_ms, err, &dQry) != 0) return -1;
    double t1 = now_ms();
    // --- Reduce on the device for frames with more chunks than ChunksPerFrame
    std::vector<int> red_idx, Ns;
    std::vector<int64_t> red_xoff;
    std::vector<char> is_red(size_t(nfr), 0);
    for (int i = 0; i < nfr; ++i)
        if (opt_.precision > 0 && frames[i].n > K) {
            red_idx.push_back(i);
            Ns.push_back(frames[i].n);
            red_xoff.push_back(feat_off[i]);
            is_red[size_t(i)] = 1;
        }
    const int nred = int(red_idx.size());
    double yak_ms = 0, scan_ms = 0;
    long long passes = 0, slow = 0, restarts = 0;
    // --- the KNNFit / prune / packing pipeline's slabs (whole range, allocated
    // before the scan starts: nothing is allocated or freed while it runs)
    // the shared pinned arena is held for the whole encode, and released only
    // after pc's stream and every device launch of this encode have drained
    // (members are destroyed in reverse order: drain, pc, then the lock)
    PinnedArena& pa = pinned_arena();
    std::lock_guard<std::mutex> arena_lock(pa.m);
    struct DeviceDrain {
        ~DeviceDrain() { (void)hipDeviceSynchronize(); }
    } drain_before_unlock;
    PostCtx pc;
    pc.recon = recon != nullptr;
    pc.dQry = dQry.p;
    pc.coff.resize(size_t(nfr));
    pc.roff.resize(size_t(nfr));
    pc.woff.resize(size_t(nfr));
    pc.noff.resize(size_t(nfr));
    int64_t nc = 0, nr = 0, nw = 0, nn = 0;
    for (int i = 0; i < nfr; ++i) {
        const int rmax = is_red[size_t(i)] ? K : frames[i].n;  // reducedChunks.Count before pruning
        pc.coff[size_t(i)] = nc;
        pc.roff[size_t(i)] = nr;
        pc.woff[size_t(i)] = nw;
        pc.noff[size_t(i)] = nn;
        nc += int64_t(rmax) * cs;
        nr += rmax;
        nw += pack_word_capacity(frames[i].n);
        nn += frames[i].n;
    }
    int64_t nred_pts = 0;
    for (int n : Ns) nred_pts += n;
    {
        auto chk = [&](hipError_t r, const char* what) {
            if (r == hipSuccess) return true;
            *err = std::string("KNNFit/pack pipeline setup: ") + what + ": " + hipGetErrorString(r);
            return false;
        };
        if (!chk(hipStreamCreateWithFlags(&pc.st, hipStreamNonBlocking), "stream") ||
            !chk(pc.dCand.alloc(size_t(nc)), "alloc") || !chk(pc.dBest.alloc(size_t(nn)), "alloc") ||
            !chk(pc.dCnt.alloc(size_t(nr)), "alloc") || !chk(pc.dRemap.alloc(size_t(nr)), "alloc") ||
            !chk(pc.dWords.alloc(size_t(nw)), "alloc") || !chk(pc.dFit.alloc(size_t(std::max(nfr, 1))), "alloc") ||
            !chk(pc.dPack.alloc(size_t(std::max(nfr, 1))), "alloc") ||
            (pc.recon && !chk(pc.dCodes.alloc(size_t(nn)), "alloc")) ||
            !chk(pa.cand.reserve(sizeof(float) * size_t(nc)), "pinned alloc") ||
            !chk(pa.cnt.reserve(sizeof(int) * size_t(nr)), "pinned alloc") ||
            !chk(pa.remap.reserve(sizeof(int) * size_t(nr)), "pinned alloc") ||
            !chk(pa.words.reserve(sizeof(uint32_t) * size_t(nw)), "pinned alloc") ||
            (pc.recon && !chk(pa.codes.reserve(sizeof(uint32_t) * size_t(nn)), "pinned alloc")) ||
            !chk(pa.cl.reserve(sizeof(int) * size_t(std::max<int64_t>(nred_pts, 1))), "pinned alloc") ||
            !chk(pa.notify.reserve(sizeof(int) * size_t(std::max(nred, 1))), "pinned alloc") ||
            !chk(hipMemsetAsync(pc.dWords.p, 0, sizeof(uint32_t) * size_t(nw), pc.st), "memset"))
            return -1;
    }
    pc.hCand = pa.cand.as<float>();
    pc.hCnt = pa.cnt.as<int>();
    pc.hRemap = pa.remap.as<int>();
    pc.hWords = pa.words.as<uint32_t>();
    pc.hCodes = pa.codes.as<uint32_t>();
    int* notify = pa.notify.as<int>();
    int* cl_host = pa.cl.as<int>();
    std::memset(notify, 0, sizeof(int) * size_t(std::max(nred, 1)));
    std::vector<int64_t> red_noff(size_t(nred) + 1, 0);  // reduced frame j's clusters at cl_host + red_noff[j]
    std::vector<int> red_pos(size_t(nfr), -1);
    for (int j = 0; j < nred; ++j) {
        red_noff[size_t(j) + 1] = red_noff[size_t(j)] + Ns[size_t(j)];
        red_pos[size_t(red_idx[size_t(j)])] = j;
    }
    // 0: scanning; 1: every frame's clusters are final (notified ones in
    // cl_host, the others in cl_final); -1: the Reduce failed
    std::atomic<int> scan_state{0};
    std::vector<int> cl_final;
    std::string post_err;
    double t_scan_end = 0, overlap_ms = 0;
    const bool batched_scan = nred > 0 && !opt_.python_reduce;
    auto post_loop = [&]() -> int {
        std::vector<char> done(size_t(nfr), 0);
        int remaining = nfr;
        while (remaining > 0) {
            const int st = scan_state.load(std::memory_order_acquire);
            if (st < 0) return 0;
            std::vector<int> ids;
            for (int i = 0; i < nfr; ++i) {
                if (done[size_t(i)]) continue;
                const int j = red_pos[size_t(i)];
                const bool notified = j >= 0 && batched_scan && __atomic_load_n(&notify[j], __ATOMIC_ACQUIRE) != 0;
                if (j < 0 || notified || st == 1) ids.push_back(i);
            }
            // during the scan, wait for a group worth a launch
            if (ids.empty() || (st == 0 && int(ids.size()) < std::min(remaining, 8))) {
                std::this_thread::sleep_for(std::chrono::microseconds(500));
                continue;
            }
            for (int i : ids) {
                const int j = red_pos[size_t(i)];
                if (j < 0 || !batched_scan) continue;
                FrameState& f = frames[size_t(i)];
                if (__atomic_load_n(&notify[j], __ATOMIC_ACQUIRE) != 0)
                    f.clusters.assign(cl_host + red_noff[size_t(j)], cl_host + red_noff[size_t(j) + 1]);
                else
                    f.clusters.assign(cl_final.begin() + long(red_noff[size_t(j)]),
                                      cl_final.begin() + long(red_noff[size_t(j) + 1]));
            }
            const double tg = now_ms();
            if (post_group(frames, ids, is_red, pc, &post_err) != 0) return -1;
            if (st == 0) overlap_ms += now_ms() - tg;
            for (int i : ids) done[size_t(i)] = 1;
            remaining -= int(ids.size());
        }
        return 0;
    };
    if (nred > 0 && opt_.python_reduce) {
        // -py: TFrame.Reduce with PythonReduce (encoder.lpr:837-841): Birch labels
        // (gsc_birch_host.cpp), no yakmo and no KNNScanReduce
        const double tb = now_ms();
        for (size_t j = 0; j < red_idx.size(); ++j) {
            FrameState& f = frames[red_idx[j]];
            std::vector<float> x(size_t(f.n) * DP);
            if (hipMemcpy(x.data(), dFeat.p + red_xoff[j], sizeof(float) * x.size(), hipMemcpyDeviceToHost) !=
                hipSuccess) {
                *err = "-py: feature download failed";
                return -1;
            }
            compact_rows(&x, f.n, DP, D);  // cluster.py reads the real features (extern.pas:363-369)
            f.clusters.resize(size_t(f.n));
            if (birch_reduce_labels(f.n, D, x.data(), K, f.clusters.data(), err) != 0) return -1;
            f.scan_iters = 0;
            f.scan_slow = 0;
        }
        scan_ms += now_ms() - tb;
    }
    int post_rc = 0;
    if (batched_scan) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        std::thread worker([&] {
            if (hipSetDevice(dev) != hipSuccess) {
                post_err = "KNNFit/pack pipeline: hipSetDevice failed";
                post_rc = -1;
                return;
            }
            post_rc = post_loop();
        });
        std::vector<float> C;
        std::vector<int> it, sl;
        g_scan_rounds.store(0);
        int* cl_dev = nullptr;
        int* nt_dev = nullptr;
        int rr = 0;
        if (hipHostGetDevicePointer(reinterpret_cast<void**>(&cl_dev), cl_host, 0) != hipSuccess ||
            hipHostGetDevicePointer(reinterpret_cast<void**>(&nt_dev), notify, 0) != hipSuccess) {
            rr = fail("KNNScanReduce: no device address for the host-mapped cluster buffers");
        } else {
            rr = run_reduce_batch_dev(DP, K, opt_.precision, Ns, red_xoff, dFeat.p, &C, &cl_final, &it, &sl, &restarts,
                                      &yak_ms, &scan_ms, cl_dev, nt_dev, D);
        }
        t_scan_end = now_ms();
        if (rr != 0) *err = t_err;
        scan_state.store(rr != 0 ? -1 : 1, std::memory_order_release);
        worker.join();
        if (rr != 0) return -1;
        for (int j = 0; j < nred; ++j) {
            FrameState& f = frames[size_t(red_idx[size_t(j)])];
            f.scan_iters = it[size_t(j)];
            f.scan_slow = sl[size_t(j)];
            passes += it[size_t(j)];
            slow += sl[size_t(j)];
        }
    } else {
        t_scan_end = now_ms();
        scan_state.store(1, std::memory_order_release);
        post_rc = post_loop();
    }
    if (post_rc != 0) {
        *err = post_err;
        return -1;
    }
    const double t2 = t_scan_end;
    const double t3 = now_ms();
    if (recon && device_recon(b, frames, recon, err) != 0) return -1;
    const double recon_ms = now_ms() - t3;
    out->clear();
    size_t bytes = 0;
    for (auto& f : frames) bytes += f.stream.size();
    out->reserve(bytes);
    for (auto& f : frames) out->insert(out->end(), f.stream.begin(), f.stream.end());
    if (frame_bytes) {
        frame_bytes->clear();
        for (auto& f : frames) frame_bytes->push_back(f.stream.size());
    }
    double t4 = now_ms();
    if (std::getenv("GSC_HOST_TIMING"))
        std::fprintf(stderr,
                     "host timing [ms]: frames+dsp %.1f (dsp %.1f) | reduce (yakmo %.1f scan %.1f) %.1f |"
                     " post after the scan %.1f (in the scan tail %.1f, KNNFit kernels %.1f, %d groups) | concat %.1f"
                     " | hipMalloc/hipFree so far %.1f\n",
                     t1 - t0, dsp_ms, yak_ms, scan_ms, t2 - t1, t3 - t2, overlap_ms, pc.knn_ms, pc.groups, t4 - t3,
                     double(g_devbuf_ns.exchange(0)) / 1e6);
    if (std::getenv("GSC_HOST_TIMING") && !red_idx.empty()) {  // per-frame pass counts (scan tail)
        std::vector<int> h(kMaxScanIters + 1, 0);
        for (int i : red_idx) h[std::min(kMaxScanIters, std::max(0, frames[i].scan_iters))]++;
        std::fprintf(stderr, "scan passes histogram:");
        for (int v = 0; v <= kMaxScanIters; ++v)
            if (h[v]) std::fprintf(stderr, " %d:%d", v, h[v]);
        std::fprintf(stderr, "\n");
    }
    if (tim) {
        tim->host_frames_ms = t1 - t0 - dsp_ms;
        tim->gpu_dsp_ms = dsp_ms;
        tim->gpu_yakmo_ms = yak_ms;
        tim->gpu_scan_ms = scan_ms;
        tim->gpu_knnfit_ms = pc.knn_ms;
        tim->host_post_ms = t4 - t2 - recon_ms;  // what the post-processing adds after the scan
        tim->gpu_recon_ms = recon_ms;
        tim->post_overlap_ms = overlap_ms;
        tim->post_groups = pc.groups;
        tim->knnfit_overflow = pc.ov_queries;
        tim->frames = nfr;
        tim->reduce_frames = int(red_idx.size());
        long long pts = 0;
        for (auto& f : frames) pts += f.n;
        tim->points = pts;
        tim->scan_passes = passes;
        tim->scan_slow = slow;
        tim->scan_restarts = restarts;
        long long pp = 0;
        for (auto& f : frames) pp += (long long)f.scan_iters * f.n;
        tim->scan_point_passes = pp;
        tim->scan_launches = g_scan_rounds.exchange(0);
        tim->knnfit_launches = pc.groups;
        long long cand = 0;
        for (auto& f : frames) cand += (long long)f.n * 4 * f.r_before_prune;
        tim->knnfit_pairs = cand;
    }
    return 0;
}

}  // namespace gsc

// ============================================================================
// C ABI
// ============================================================================
using namespace gsc;

extern "C" {

void gsc_default_options(gsc_options* o) {
    std::memset(o, 0, sizeof(*o));
    o->bit_rate = -1;
    o->precision = 3;
    o->low_cut = 0.0;
    o->high_cut = 24000.0;
    o->chunk_bit_depth = 8;
    o->chunk_size = 4;
    o->chunks_per_frame = 4096;
    o->reduce_bass_band = 1;
    o->vfr = 1.0;
    o->chunk_blend = 0;
    o->frame_length = 4000.0;
}

static int opt_start(int argc, const char* const* argv, const char* pfx) {
    const size_t l = std::strlen(pfx);
    for (int i = 0; i < argc; ++i)
        if (std::strncmp(argv[i], pfx, l) == 0) return i;
    return -1;
}
static double opt_value(int argc, const char* const* argv, const char* pfx, double def) {
    const int i = opt_start(argc, argv, pfx);
    if (i < 0) return def;
    const char* s = argv[i] + std::strlen(pfx);
    if (!*s) return def;
    char* end = nullptr;
    const double v = std::strtod(s, &end);
    return (end && !*end) ? v : def;  // StrToFloatDef
}
static bool opt_has(int argc, const char* const* argv, const char* p) {
    for (int i = 0; i < argc; ++i)
        if (strcasecmp(argv[i], p) == 0) return true;
    return false;
}

void gsc_parse_options(gsc_options* o, int argc, const char* const* argv) {
    auto clampi = [](int64_t v, int64_t lo, int64_t hi) { return int(std::min(hi, std::max(lo, v))); };
    o->bit_rate = int(fpc::round(opt_value(argc, argv, "-br", o->bit_rate)));
    o->precision = int(fpc::round(opt_value(argc, argv, "-pr", o->precision)));
    o->low_cut = opt_value(argc, argv, "-lc", o->low_cut);
    o->high_cut = opt_value(argc, argv, "-hc", o->high_cut);
    o->vfr = std::min(1.0, std::max(0.0, opt_value(argc, argv, "-vfr", o->vfr)));
    o->frame_length = std::max(opt_value(argc, argv, "-fl", o->frame_length), 1.0);
    o->chunk_bit_depth = clampi(fpc::round(opt_value(argc, argv, "-cbd", o->chunk_bit_depth)), 1, 16);
    o->chunk_size = int(fpc::round(opt_value(argc, argv, "-cs", o->chunk_size)));
    o->chunks_per_frame = clampi(fpc::round(opt_value(argc, argv, "-cpf", o->chunks_per_frame)), 256, 4096);
    o->verbose = opt_has(argc, argv, "-v");
    o->reduce_bass_band = !opt_has(argc, argv, "-pbb");
    o->chunk_blend = clampi(fpc::round(opt_value(argc, argv, "-cb", o->chunk_blend)), 0, o->chunk_size / 2);
    o->python_reduce = opt_has(argc, argv, "-py");
}

int gsc_count_frames(const uint8_t* wav, size_t wav_len, const gsc_options* o, int* frame_count) {
    Encoder enc(*o);
    std::string err;
    if (enc.prepare(wav, wav_len, &err) != 0) return fail(err);
    *frame_count = enc.frame_count();
    return 0;
}

// encode frames [frame_begin, frame_end) of a prepared encoder into a
// library-allocated buffer; timing lands in t_tim (host_prepare_ms excluded).
// file_bytes: the range's bytes of every file of the batch; frame_bytes: each
// frame's SaveStream bytes (frame_end - frame_begin entries)
static int encode_prepared(Encoder& enc, int frame_begin, int frame_end, uint8_t** out, size_t* out_len,
                           size_t* file_bytes = nullptr, size_t* frame_bytes = nullptr) {
    const double t0 = now_ms();
    const int fc = enc.frame_count();
    frame_begin = std::max(0, frame_begin);
    frame_end = std::min(fc, frame_end < 0 ? fc : frame_end);
    std::vector<uint8_t> bytes;
    std::vector<size_t> fb;
    std::string err;
    if (frame_end > frame_begin) {
        if (enc.encode_range(frame_begin, frame_end, &bytes, &err, &t_tim, nullptr, &fb) != 0) return fail(err);
    }
    if (file_bytes) {
        const std::vector<int>& ff = enc.file_first();
        for (size_t f = 0; f + 1 < ff.size(); ++f) {
            size_t n = 0;
            for (int i = std::max(ff[f], frame_begin); i < std::min(ff[f + 1], frame_end); ++i)
                n += fb[size_t(i - frame_begin)];
            file_bytes[f] = n;
        }
    }
    if (frame_bytes)
        for (int i = frame_begin; i < frame_end; ++i) frame_bytes[i - frame_begin] = fb[size_t(i - frame_begin)];
    *out = static_cast<uint8_t*>(std::malloc(std::max<size_t>(bytes.size(), 1)));
    if (!*out) return fail("out of host memory");
    if (!bytes.empty()) std::memcpy(*out, bytes.data(), bytes.size());
    *out_len = bytes.size();
    t_tim.total_ms = now_ms() - t0;
    return 0;
}

int gsc_encode_wav_frames(const uint8_t* wav, size_t wav_len, const gsc_options* o, int frame_begin, int frame_end,
                          uint8_t** out, size_t* out_len, int* frame_count) {
    const double t0 = now_ms();
    t_tim = gsc_timing{};
    Encoder enc(*o);
    std::string err;
    if (enc.prepare(wav, wav_len, &err) != 0) return fail(err);
    const double t1 = now_ms();
    if (frame_count) *frame_count = enc.frame_count();
    if (encode_prepared(enc, frame_begin, frame_end, out, out_len) != 0) return -1;
    t_tim.host_prepare_ms = t1 - t0;
    t_tim.total_ms = now_ms() - t0;
    return 0;
}

}  // extern "C"

// a WAV after Load + PrepareFrames: the frame boundaries of the whole file,
// computed once per job and shared by every frame-range encode (sharding)
struct gsc_prepared {
    Encoder enc;
    double prepare_ms = 0;
    int loaded_begin = 0, loaded_end = -1;  // frames whose samples are held (-1: all)
    explicit gsc_prepared(const gsc_options& o) : enc(o) {}
};

extern "C" {

gsc_prepared* gsc_prepare(const uint8_t* wav, size_t wav_len, const gsc_options* o) {
    if (!wav || !o) {
        fail("gsc_prepare: null argument");
        return nullptr;
    }
    const double t0 = now_ms();
    gsc_prepared* p = new (std::nothrow) gsc_prepared(*o);
    if (!p) {
        fail("gsc_prepare: out of host memory");
        return nullptr;
    }
    std::string err;
    if (p->enc.prepare(wav, wav_len, &err) != 0) {
        delete p;
        fail(err);
        return nullptr;
    }
    p->prepare_ms = now_ms() - t0;
    return p;
}

int gsc_prepared_frame_count(const gsc_prepared* p) { return p ? p->enc.frame_count() : -1; }

int gsc_prepared_frame_chunks(const gsc_prepared* p, int* chunks) {
    if (!p || !chunks) return fail("gsc_prepared_frame_chunks: null argument");
    for (int i = 0; i < p->enc.frame_count(); ++i) chunks[i] = p->enc.frame_chunks(i);
    return 0;
}

int gsc_prepared_frame_bounds(const gsc_prepared* p, int* starts, int* ends) {
    if (!p || !starts || !ends) return fail("gsc_prepared_frame_bounds: null argument");
    const auto& s = p->enc.frame_starts();
    const auto& e = p->enc.frame_ends();
    std::copy(s.begin(), s.end(), starts);
    std::copy(e.begin(), e.end(), ends);
    return 0;
}

gsc_prepared* gsc_prepare_frames(const uint8_t* wav, size_t wav_len, const gsc_options* o, const int* starts,
                                 const int* ends, int frame_count, int frame_begin, int frame_end) {
    if (!wav || !o || !starts || !ends) {
        fail("gsc_prepare_frames: null argument");
        return nullptr;
    }
    const double t0 = now_ms();
    gsc_prepared* p = new (std::nothrow) gsc_prepared(*o);
    if (!p) {
        fail("gsc_prepare_frames: out of host memory");
        return nullptr;
    }
    std::string err;
    if (frame_end < 0) frame_end = frame_count;
    if (p->enc.prepare_bounds(wav, wav_len, starts, ends, frame_count, frame_begin, frame_end, &err) != 0) {
        delete p;
        fail(err);
        return nullptr;
    }
    p->loaded_begin = frame_begin;
    p->loaded_end = frame_end;
    p->prepare_ms = now_ms() - t0;
    return p;
}

// every prepared entry point: a bounds-prepared encoder (gsc_prepare_frames)
// holds only the samples of frames [loaded_begin, loaded_end)
static int check_loaded(const gsc_prepared* p, int frame_begin, int frame_end, const char* who) {
    if (p->loaded_end < 0) return 0;
    const int fe = frame_end < 0 ? p->enc.frame_count() : std::min(frame_end, p->enc.frame_count());
    const int fb = std::max(0, frame_begin);
    if (fe > fb && (fb < p->loaded_begin || fe > p->loaded_end))
        return fail(std::string(who) + ": frames outside the range gsc_prepare_frames loaded");
    return 0;
}

int gsc_encode_prepared(gsc_prepared* p, int frame_begin, int frame_end, uint8_t** out, size_t* out_len) {
    return gsc_encode_prepared_frames(p, frame_begin, frame_end, out, out_len, nullptr);
}

int gsc_encode_prepared_frames(gsc_prepared* p, int frame_begin, int frame_end, uint8_t** out, size_t* out_len,
                               size_t* frame_bytes) {
    if (!p || !out || !out_len) return fail("gsc_encode_prepared: null argument");
    if (check_loaded(p, frame_begin, frame_end, "gsc_encode_prepared") != 0) return -1;
    t_tim = gsc_timing{};
    if (encode_prepared(p->enc, frame_begin, frame_end, out, out_len, nullptr, frame_bytes) != 0) return -1;
    t_tim.host_prepare_ms = 0;  // paid once, in gsc_prepare
    return 0;
}

double gsc_prepared_prepare_ms(const gsc_prepared* p) { return p ? p->prepare_ms : 0.0; }

gsc_prepared* gsc_prepare_many(const uint8_t* const* wavs, const size_t* lens, int nfiles, const gsc_options* o) {
    if (!wavs || !lens || !o || nfiles <= 0) {
        fail("gsc_prepare_many: invalid argument");
        return nullptr;
    }
    const double t0 = now_ms();
    gsc_prepared* p = new (std::nothrow) gsc_prepared(*o);
    if (!p) {
        fail("gsc_prepare_many: out of host memory");
        return nullptr;
    }
    std::string err;
    if (p->enc.prepare_many(wavs, lens, nfiles, &err) != 0) {
        delete p;
        fail(err);
        return nullptr;
    }
    p->prepare_ms = now_ms() - t0;
    return p;
}

int gsc_prepared_file_count(const gsc_prepared* p) { return p ? int(p->enc.file_first().size()) - 1 : -1; }

int gsc_prepared_file_frames(const gsc_prepared* p, int* first_frame) {
    if (!p || !first_frame) return fail("gsc_prepared_file_frames: null argument");
    const auto& ff = p->enc.file_first();
    std::copy(ff.begin(), ff.end(), first_frame);
    return 0;
}

int gsc_encode_prepared_files(gsc_prepared* p, int frame_begin, int frame_end, uint8_t** out, size_t* out_len,
                              size_t* file_bytes) {
    if (!p || !out || !out_len || !file_bytes) return fail("gsc_encode_prepared_files: null argument");
    if (check_loaded(p, frame_begin, frame_end, "gsc_encode_prepared_files") != 0) return -1;
    t_tim = gsc_timing{};
    if (encode_prepared(p->enc, frame_begin, frame_end, out, out_len, file_bytes) != 0) return -1;
    return 0;
}

void gsc_prepared_free(gsc_prepared* p) { delete p; }

int gsc_frame_dsp(const uint8_t* wav, size_t wav_len, const gsc_options* o, int frame, int* atten_div, float** feat,
                  int* n_chunks) {
    Encoder enc(*o);
    std::string err;
    if (enc.prepare(wav, wav_len, &err) != 0) return fail(err);
    std::vector<float> f;
    if (enc.dsp_frame(frame, atten_div, &f, &err) != 0) return fail(err);
    *n_chunks = int(f.size() / size_t(2 * o->chunk_size));
    *feat = static_cast<float*>(std::malloc(std::max<size_t>(f.size(), 1) * sizeof(float)));
    if (!f.empty()) std::memcpy(*feat, f.data(), f.size() * sizeof(float));
    return 0;
}

int gsc_encode_wav(const uint8_t* wav, size_t wav_len, const gsc_options* o, uint8_t** out, size_t* out_len) {
    return gsc_encode_wav_frames(wav, wav_len, o, 0, -1, out, out_len, nullptr);
}

int gsc_encode_wav_recon(const uint8_t* wav, size_t wav_len, const gsc_options* o, uint8_t** out, size_t* out_len,
                         int16_t** recon, size_t* recon_len, double* psy_a_delta) {
    if (!wav || !o || !out || !out_len || !recon || !recon_len || !psy_a_delta)
        return fail("gsc_encode_wav_recon: null argument");
    *out = nullptr;
    *recon = nullptr;
    t_tim = gsc_timing{};
    const double t0 = now_ms();
    Encoder enc(*o);
    std::string err;
    if (enc.prepare(wav, wav_len, &err) != 0) return fail(err);
    t_tim.host_prepare_ms = now_ms() - t0;
    const int ch = enc.channels();
    const size_t n = size_t(enc.sample_count()) * size_t(ch);
    ReconOut ro;
    ro.pcm = static_cast<int16_t*>(std::calloc(std::max<size_t>(n, 1), sizeof(int16_t)));
    if (!ro.pcm) return fail("out of host memory");
    ro.wav = wav;
    ro.wav_len = wav_len;
    std::vector<uint8_t> bytes;
    const int fc = enc.frame_count();
    if (fc > 0 && enc.encode_range(0, fc, &bytes, &err, &t_tim, &ro) != 0) {
        std::free(ro.pcm);
        return fail(err);
    }
    *out = static_cast<uint8_t*>(std::malloc(std::max<size_t>(bytes.size(), 1)));
    if (!*out) {
        std::free(ro.pcm);
        return fail("out of host memory");
    }
    if (!bytes.empty()) std::memcpy(*out, bytes.data(), bytes.size());
    *out_len = bytes.size();
    // ComputePsyADelta = CompareEuclidean over Double copies (encoder.lpr:1803-1814,1862-1880): every
    // partial sum is an integer, exact in f64 below 2^53, where it equals the device's exact sum
    double acc = 0.0;
    if (ro.sq < (1ull << 53)) {
        acc = double(ro.sq);
    } else {  // the reference's sequential f64 sum, channel-major
        const size_t psc = wav_len >= 44 ? (wav_len - 44) / (2 * size_t(ch)) : 0;
        for (int j = 0; j < ch; ++j)
            for (size_t i = 0; i < size_t(enc.sample_count()); ++i) {
                int16_t sv = 0;
                if (i < psc) std::memcpy(&sv, wav + 44 + (i * ch + j) * 2, 2);
                const double d = double(sv) - double(ro.pcm[i * ch + j]);
                acc += d * d;
            }
    }
    *psy_a_delta = n ? std::sqrt(acc / double(n)) : 0.0;
    *recon = ro.pcm;
    *recon_len = n;
    t_tim.total_ms = now_ms() - t0;
    return 0;
}

// rows of d floats -> rows of dp (trailing zeros)
static std::vector<float> pad_rows(const float* x, int n, int d, int dp) {
    std::vector<float> v(size_t(n) * dp, 0.0f);
    for (int i = 0; i < n; ++i) std::memcpy(&v[size_t(i) * dp], x + size_t(i) * d, sizeof(float) * size_t(d));
    return v;
}

extern "C" hipError_t gsc_launch_yakmo_chain_test(int ppl, const float* pts, int nbk, float run, int* k_out,
                                                  float* out);

int gsc_yakmo_chain_test(int ppl, const float* pts, int nbk, float run, int* accepted, float* run_out, float* ck,
                         float* bmn, float* bmx) {
    if (ensure_device() != 0) return -1;
    if ((ppl != 8 && ppl != 16) || nbk < 1 || nbk > ppl) return fail("gsc_yakmo_chain_test: ppl 8 / 16, 1 <= nbk <= ppl");
    DevBuf<float> dP, dO;
    DevBuf<int> dK;
    HIP_TRY(dP.alloc(size_t(64) * nbk));
    HIP_TRY(dO.alloc(1 + 3 * 64));
    HIP_TRY(dK.alloc(1));
    HIP_TRY(hipMemcpy(dP.p, pts, sizeof(float) * 64 * size_t(nbk), hipMemcpyHostToDevice));
    HIP_TRY(gsc_launch_yakmo_chain_test(ppl, dP.p, nbk, run, dK.p, dO.p));
    HIP_TRY(hipDeviceSynchronize());
    float o[1 + 3 * 64];
    HIP_TRY(hipMemcpy(o, dO.p, sizeof(o), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(accepted, dK.p, sizeof(int), hipMemcpyDeviceToHost));
    *run_out = o[0];
    for (int b = 0; b < nbk; ++b) {
        ck[b] = o[1 + b];
        bmn[b] = o[1 + 64 + b];
        bmx[b] = o[1 + 128 + b];
    }
    return 0;
}

int gsc_yakmo_seed_means(int n, int d0, const float* x, int k, float* centroids) {
    if (ensure_device() != 0) return -1;
    if (k >= n || k <= 0 || k > kMaxK) return fail("yakmo needs 0 < k < n, k <= 4096");
    if (d0 <= 0 || d0 > 32) return fail("yakmo: 1 <= d <= 32 features");
    const int d = feature_stride((d0 + 1) / 2);  // the kernel width; trailing zero features change nothing
    std::vector<float> X = pad_rows(x, n, d0, d), C;
    std::vector<int> cl, it, sl;
    // run only the seeding part: precision 0 => scan loop still runs once; use a
    // dedicated path instead
    const int nf = 1;
    std::vector<ReduceFrame> fr(1);
    fr[0] = ReduceFrame{};
    fr[0].N = n;
    fr[0].K = k;
    fr[0].k_off = n;
    DevBuf<float> dX, dC, dF, dYSum;
    DevBuf<int> dI;
    DevBuf<uint32_t> dBits;
    DevBuf<ReduceFrame> dFr;
    HIP_TRY(dX.alloc(X.size()));
    HIP_TRY(dC.alloc(size_t(k) * d));
    HIP_TRY(dF.alloc(size_t(n) * 4));
    HIP_TRY(dI.alloc(size_t(n) + size_t(k)));
    HIP_TRY(dBits.alloc(gsc_yakmo_big_words(n, 1)));
    HIP_TRY(dYSum.alloc(gsc_yakmo_big_floats(n, 1)));
    HIP_TRY(dFr.alloc(1));
    HIP_TRY(hipMemcpy(dX.p, X.data(), sizeof(float) * X.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dFr.p, fr.data(), sizeof(ReduceFrame), hipMemcpyHostToDevice));
    HIP_TRY(gsc_launch_yakmo(d, dFr.p, nf, dX.p, dC.p, dF.p, dI.p, dYSum.p, dBits.p, n, nullptr));
    HIP_TRY(hipDeviceSynchronize());
    C.resize(size_t(k) * d);
    HIP_TRY(hipMemcpy(C.data(), dC.p, sizeof(float) * size_t(k) * d, hipMemcpyDeviceToHost));
    compact_rows(&C, k, d, d0);
    std::memcpy(centroids, C.data(), sizeof(float) * size_t(k) * d0);
    (void)cl;
    (void)it;
    (void)sl;
    return 0;
}

int gsc_scan_reduce(int n, int d0, const float* x, int k, float* centroids, int* clusters, int precision, int* iters) {
    if (ensure_device() != 0) return -1;
    // same kernels as the encoder, but starting from caller-provided centroids:
    // seed via yakmo is skipped by uploading the centroids after the yakmo launch
    if (d0 <= 0 || d0 > 32) return fail("KNNScanReduce kernels support 1 <= d <= 32 features");
    const int d = feature_stride((d0 + 1) / 2);  // padded with zero features (residual divides by d0)
    const std::vector<float> xp = pad_rows(x, n, d0, d);
    std::vector<float> cp = pad_rows(centroids, k, d0, d);
    x = xp.data();
    std::vector<ReduceFrame> fr(1);
    fr[0] = ReduceFrame{};
    fr[0].N = n;
    fr[0].K = k;
    fr[0].dcol = d0;
    fr[0].k_off = n;
    fr[0].ka_off = n + k;
    DevBuf<float> dX, dC, dRate, dF;
    DevBuf<int> dI;
    DevBuf<ReduceFrame> dFr;
    HIP_TRY(dF.alloc(size_t(n) * 4));
    HIP_TRY(dX.alloc(size_t(n) * d));
    HIP_TRY(dC.alloc(size_t(k) * d));
    HIP_TRY(dI.alloc(size_t(n) + size_t(k) + size_t(padded_k(k))));
    HIP_TRY(dFr.alloc(1));
    const std::vector<float> rt = rate_table(n);
    HIP_TRY(dRate.alloc(rt.size()));
    HIP_TRY(hipMemcpy(dX.p, x, sizeof(float) * size_t(n) * d, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dC.p, cp.data(), sizeof(float) * size_t(k) * d, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dRate.p, rt.data(), sizeof(float) * rt.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dFr.p, fr.data(), sizeof(ReduceFrame), hipMemcpyHostToDevice));
    HIP_TRY(launch_scan_passes(d, dFr.p, 1, k, dX.p, dC.p, dI.p, dF.p, dRate.p, precision));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(cp.data(), dC.p, sizeof(float) * size_t(k) * d, hipMemcpyDeviceToHost));
    compact_rows(&cp, k, d, d0);
    std::memcpy(centroids, cp.data(), sizeof(float) * size_t(k) * d0);
    HIP_TRY(hipMemcpy(clusters, dI.p, sizeof(int) * size_t(n), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(fr.data(), dFr.p, sizeof(ReduceFrame), hipMemcpyDeviceToHost));
    if (iters) *iters = fr[0].iters;
    if (fr[0].loop_iters < 0) return fail("KNNScanReduce: batched pipeline made no progress (guard tripped)");
    if (std::getenv("GSC_SCAN_DEBUG"))
    {
        std::fprintf(stderr, "scan: passes %d slow %d restarts %d loop_iters(last pass) %d err %.9g tree_exact %d\n",
                     fr[0].iters, fr[0].slow, fr[0].restarts, fr[0].loop_iters, fr[0].err, fr[0].tree_exact);
        std::fprintf(stderr, "stamps [prep A1 A2 B2 part3 part4 B1 vcheck won setup soloA soloDFS a2win a2far a2box a2out]");
        for (int w = 0; w < 8; ++w) {
            std::fprintf(stderr, "\n  w%d:", w);
            for (int k = 0; k < 16; ++k) std::fprintf(stderr, " %.3g", double(fr[0].stamps[w * 16 + k]));
        }
        std::fprintf(stderr, "\nA1 queries [home pruned evaluated | iterations fixups pending | clk: box+home midbarrier]"
                             "\n  (one-CU frames: stamps slot 'vcheck' = A1 after the mid barrier + vp_end, slot 'A1' = the V check)");
        for (int w = 0; w < 8; ++w) {
            std::fprintf(stderr, "\n  w%d:", w);
            for (int k = 0; k < 8; ++k) std::fprintf(stderr, " %.4g", double(fr[0].acounts[w * 8 + k]));
        }
        const uint64_t* x = fr[0].xcounts;
        std::fprintf(stderr,
                     "\niterations [kind: count, cycles]: bubble %llu %.4g | with new queries %llu %.4g (new queries %llu)"
                     " | with fixups %llu %.4g | with a solo %llu %.4g | A2 queries on per-wave bounds %llu",
                     (unsigned long long)x[0], double(x[1]), (unsigned long long)x[2], double(x[3]),
                     (unsigned long long)x[8], (unsigned long long)x[4], double(x[5]), (unsigned long long)x[6],
                     double(x[7]), (unsigned long long)x[9]);
        std::fprintf(stderr, "\napproximate certificates failed: no unique minimum %llu, a far step not provable %llu",
                     (unsigned long long)x[10], (unsigned long long)x[11]);
        std::fprintf(stderr, "\nfailed queries by cause: snapshot uncertified %llu, c* moved past m2 %llu, V check %llu"
                     " (V check only %llu)", (unsigned long long)x[12], (unsigned long long)x[13],
                     (unsigned long long)x[14], (unsigned long long)x[15]);
        const uint64_t* x2 = fr[0].xcounts2;
        std::fprintf(stderr, "\nsolo answer = speculative c*: by cause uncertified %llu, m2 %llu, V %llu | solos with a remainder"
                             " %llu, of them same answer %llu (remainder queries valid to the next failure %llu, whole"
                             " remainder valid %llu)", (unsigned long long)x2[0], (unsigned long long)x2[1],
                     (unsigned long long)x2[2], (unsigned long long)x2[3], (unsigned long long)x2[4],
                     (unsigned long long)x2[5], (unsigned long long)x2[6]);
        std::fprintf(stderr, "\nin-batch DFS answers %llu, of them failing at commit %llu", (unsigned long long)x2[8],
                     (unsigned long long)x2[9]);
        std::fprintf(stderr, "\n");
    }
    return 0;
}

int gsc_birch_labels(int n, int d, const float* x, int k, int* labels) {
    if (!x || !labels || n <= 0 || d <= 0 || k <= 0) return fail("gsc_birch_labels: invalid argument");
    if (ensure_device() != 0) return -1;
    std::string err;
    if (birch_reduce_labels(n, d, x, k, labels, &err) != 0) return fail(err);
    return 0;
}

int gsc_knnfit_assign(int r, int cs, const float* cand_fwd, int n, const float* q, float eps, int* best) {
    if (ensure_device() != 0) return -1;
    std::vector<int> Rs{r}, Ns{n}, out;
    std::vector<float> E{eps}, C(cand_fwd, cand_fwd + size_t(r) * cs), Q(q, q + size_t(n) * cs);
    double ms = 0;
    if (run_knnfit_batch(cs, Rs, Ns, E, C, Q, &out, &ms) != 0) return -1;
    std::memcpy(best, out.data(), sizeof(int) * size_t(n));
    return 0;
}

void gsc_last_timing(gsc_timing* t) { *t = t_tim; }

int gsc_set_device(int device) {
    HIP_TRY(hipSetDevice(device));
    return 0;
}

int gsc_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* gsc_last_error(void) { return t_err.c_str(); }

void gsc_free(void* p) { std::free(p); }

}  // extern "C"
