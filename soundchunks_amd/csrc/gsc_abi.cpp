// The extern.pas:112-123 drop-in surface (yakmo_single.dll + ANN.dll exports)
// implemented on the GPU.  Semantics follow the DLLs as the reference uses
// them: yakmo copies its training rows; ANN keeps the caller's row pointers
// and every search reads the points' *current* values (KNNScanReduce relies on
// that, encoder.lpr:729-745), so each search stages the live rows.
//
// Errors.  The reference signatures have no error channel (the DLLs return no
// codes; a Pascal caller indexes Centroids[idx] with whatever a search
// returns, encoder.lpr:733-739).  So a device failure inside a search or a
// yakmo call is fatal: the library prints what failed and aborts, instead of
// returning an index the caller would dereference.  ann_kdtree_create returns
// NULL when the device is unusable or allocation fails (every buffer it got is
// freed); passing NULL to a search aborts too.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/soundchunks.h"
#include "gsc_device.h"

extern "C" hipError_t gsc_launch_yakmo(int D, const gsc::ReduceFrame* frames, int nframes, const float* X, float* C,
                                       float* fs, int* is, float* gsum, uint32_t* gbits, int max_n, hipStream_t st);
extern "C" size_t gsc_yakmo_big_floats(int64_t total_points, int nframes);
extern "C" size_t gsc_yakmo_big_words(int64_t total_points, int nframes);
extern "C" hipError_t gsc_launch_ann_build(const float* pts, int n, int dd, int* pidx, int* cd, float* cv, float* lo,
                                           float* hi, float* bnd, float* val, hipStream_t st);
extern "C" hipError_t gsc_launch_ann_query(const float* pts, int n, int dd, int* pidx, int* cd, float* cv, float* lo,
                                           float* hi, float* bnd, const float* q, int k, int mode, float eps,
                                           int* idxs, float* errs, float* dist, float* mk_key, int* mk_info,
                                           float* pq_key, int* pq_h, int* pq_s, int* pq_n, hipStream_t st);

namespace {

[[noreturn]] void fatal(const char* fn, const char* what) {
    std::fprintf(stderr, "soundchunks_amd: %s: %s (fatal: the reference ABI has no error channel)\n", fn, what);
    std::fflush(stderr);
    std::abort();
}

void check(const char* fn, hipError_t e) {
    if (e != hipSuccess) fatal(fn, hipGetErrorString(e));
}

template <typename T>
T* dalloc(size_t n) {
    T* p = nullptr;
    if (hipMalloc(&p, sizeof(T) * (n ? n : 1)) != hipSuccess) return nullptr;
    return p;
}

template <typename T>
void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

// device buffer freed on every exit path
template <typename T>
struct Dev {
    T* p = nullptr;
    explicit Dev(size_t n) : p(dalloc<T>(n)) {}
    ~Dev() { dfree(p); }
    Dev(const Dev&) = delete;
    Dev& operator=(const Dev&) = delete;
};

bool device_ok() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return false;
    int dev = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return false;
    return std::strncmp(p.gcnArchName, "gfx950", 6) == 0;
}

}  // namespace

struct yakmo_t {
    unsigned k = 0;
    bool supported = true;
    unsigned rows = 0, cols = 0;
    std::vector<float> data, centroids;
    std::vector<int> labels;
};

struct ann_kdtree_t {
    float** pa = nullptr;
    int n = 0, dd = 0, cap = 0;
    float* d_pts = nullptr;
    int *d_pidx = nullptr, *d_cd = nullptr;
    float *d_cv = nullptr, *d_lo = nullptr, *d_hi = nullptr, *d_bnd = nullptr;
    float* d_q = nullptr;
    float* d_dist = nullptr;  // live leaf distances of the current query
    int* d_idx = nullptr;
    float* d_err = nullptr;
    float* d_mk = nullptr;
    int* d_mki = nullptr;
    float* d_pqk = nullptr;
    int *d_pqh = nullptr, *d_pqs = nullptr, *d_pqn = nullptr;
    int kcap = 0;
    float* h_stage = nullptr;  // pinned: live rows + query, one copy per search
    int* h_out = nullptr;      // pinned: idxs | errs of the last search

    void release() {
        d_q = nullptr;  // aliases the tail of d_pts
        for (float** p : {&d_pts, &d_cv, &d_lo, &d_hi, &d_bnd, &d_dist, &d_err, &d_mk, &d_pqk}) dfree(*p);
        for (int** p : {&d_pidx, &d_cd, &d_idx, &d_mki, &d_pqh, &d_pqs, &d_pqn}) dfree(*p);
        if (h_stage) (void)hipHostFree(h_stage);
        if (h_out) (void)hipHostFree(h_out);
        h_stage = nullptr;
        h_out = nullptr;
    }
};

extern "C" {

// ---- yakmo_single.dll ------------------------------------------------------
yakmo_t* yakmo_create(unsigned int k, unsigned int restartCount, int maxIter, int initType, int initSeed,
                      int doNormalize, int isVerbose) {
    (void)isVerbose;
    yakmo_t* y = new yakmo_t();
    y->k = k;
    // the encoder's call (encoder.lpr:824): one restart, maxIter 0, k-means++,
    // fixed seeds, no normalisation -- the only configuration implemented
    y->supported = restartCount == 1 && maxIter == 0 && initType == 1 && initSeed == 0 && doNormalize == 0;
    return y;
}

void yakmo_destroy(yakmo_t* ay) { delete ay; }

void yakmo_load_train_data(yakmo_t* ay, unsigned int rowCount, unsigned int colCount, float** dataset) {
    if (!ay) fatal("yakmo_load_train_data", "null handle");
    ay->rows = rowCount;
    ay->cols = colCount;
    ay->data.resize(size_t(rowCount) * colCount);
    for (unsigned r = 0; r < rowCount; ++r) std::memcpy(&ay->data[size_t(r) * colCount], dataset[r], 4 * colCount);
}

// k-means++ seeding (App. C.1) on the GPU; pointToCluster receives the seeding
// assignment (the DLL's single Lloyd pass only relabels points -- its labels
// are overwritten by KNNScanReduce's first pass, encoder.lpr:742 -- and the
// centroids it returns are the seeding means either way)
void yakmo_train_on_data(yakmo_t* ay, int* pointToCluster) {
    static const char* fn = "yakmo_train_on_data";
    if (!ay) fatal(fn, "null handle");
    const int N = int(ay->rows), D = int(ay->cols), K = int(ay->k);
    if (!ay->supported) fatal(fn, "only yakmo_create(K,1,0,1,0,0,v) is implemented");
    if (K <= 0 || K >= N || K > gsc::kMaxK || !(D == 8 || D == 16 || D == 32))
        fatal(fn, "unsupported shape (need 0 < K < N, K <= 4096, D in {8, 16, 32})");
    if (!device_ok()) fatal(fn, "no gfx950 device (the MI355X hot path has no CPU fallback)");
    gsc::ReduceFrame fr{};
    fr.N = N;
    fr.K = K;
    fr.k_off = N;
    Dev<float> dX(ay->data.size()), dC(size_t(K) * D), dF(4 * size_t(N));
    Dev<int> dI(size_t(N) + K);
    Dev<uint32_t> dB(gsc_yakmo_big_words(N, 1));
    Dev<float> dS(gsc_yakmo_big_floats(N, 1));
    Dev<gsc::ReduceFrame> dFr(1);
    if (!dX.p || !dC.p || !dF.p || !dI.p || !dB.p || !dS.p || !dFr.p) fatal(fn, "device allocation failed");
    check(fn, hipMemcpy(dX.p, ay->data.data(), 4 * ay->data.size(), hipMemcpyHostToDevice));
    check(fn, hipMemcpy(dFr.p, &fr, sizeof(fr), hipMemcpyHostToDevice));
    check(fn, gsc_launch_yakmo(D, dFr.p, 1, dX.p, dC.p, dF.p, dI.p, dS.p, dB.p, N, nullptr));
    ay->centroids.resize(size_t(K) * D);
    ay->labels.resize(size_t(N));
    check(fn, hipMemcpy(ay->centroids.data(), dC.p, 4 * ay->centroids.size(), hipMemcpyDeviceToHost));
    check(fn, hipMemcpy(ay->labels.data(), dI.p, 4 * size_t(N), hipMemcpyDeviceToHost));
    if (pointToCluster) std::memcpy(pointToCluster, ay->labels.data(), 4 * size_t(N));
}

void yakmo_get_centroids(yakmo_t* ay, float** centroids) {
    if (!ay) fatal("yakmo_get_centroids", "null handle");
    if (ay->centroids.size() != size_t(ay->k) * ay->cols) fatal("yakmo_get_centroids", "train_on_data has not run");
    for (unsigned c = 0; c < ay->k; ++c) std::memcpy(centroids[c], &ay->centroids[size_t(c) * ay->cols], 4 * ay->cols);
}

// ---- ANN.dll -----------------------------------------------------------------
// live rows + query into the pinned stage, one host->device copy
static void stage_points(ann_kdtree_t* t, const float* q, const char* fn) {
    const size_t nd = size_t(t->n) * size_t(t->dd);
    for (int i = 0; i < t->n; ++i) std::memcpy(t->h_stage + size_t(i) * t->dd, t->pa[i], 4 * size_t(t->dd));
    if (q) std::memcpy(t->h_stage + nd, q, 4 * size_t(t->dd));
    check(fn, hipMemcpy(t->d_pts, t->h_stage, 4 * (nd + (q ? size_t(t->dd) : 0)), hipMemcpyHostToDevice));
}

ann_kdtree_t* ann_kdtree_create(float** pa, int n, int dd, int bs, int split) {
    static const char* fn = "ann_kdtree_create";
    if (bs != 1 || split != 0 || n < 0 || dd <= 0 || (n > 0 && !pa)) return nullptr;  // only bs = 1, ANN_KD_STD
    if (!device_ok()) {
        std::fprintf(stderr, "soundchunks_amd: %s: no gfx950 device (no CPU fallback)\n", fn);
        return nullptr;
    }
    ann_kdtree_t* t = new ann_kdtree_t();
    auto give_up = [&](const char* why, hipError_t e) -> ann_kdtree_t* {
        std::fprintf(stderr, "soundchunks_amd: %s: %s: %s\n", fn, why, hipGetErrorString(e));
        (void)hipGetLastError();  // do not leave the failure to the next launch check
        t->release();
        delete t;
        return nullptr;
    };
    t->pa = pa;
    t->n = n;
    t->dd = dd;
    int p2 = 1;
    while (p2 < (n > 0 ? n : 1)) p2 <<= 1;
    t->cap = 2 * p2;
    // d_pts holds the n live rows followed by the query (d_q points into it)
    t->d_pts = dalloc<float>((size_t(n) + 1) * dd);
    t->d_pidx = dalloc<int>(size_t(n));
    t->d_cd = dalloc<int>(size_t(t->cap));
    t->d_cv = dalloc<float>(size_t(t->cap));
    t->d_lo = dalloc<float>(size_t(t->cap));
    t->d_hi = dalloc<float>(size_t(t->cap));
    t->d_bnd = dalloc<float>(2 * size_t(dd));
    t->d_dist = dalloc<float>(size_t(n));
    t->d_pqk = dalloc<float>(size_t(n) + 2);
    t->d_pqh = dalloc<int>(size_t(n) + 2);
    t->d_pqs = dalloc<int>(size_t(n) + 2);
    t->d_pqn = dalloc<int>(size_t(n) + 2);
    if (!t->d_pts || !t->d_pidx || !t->d_cd || !t->d_cv || !t->d_lo || !t->d_hi || !t->d_bnd || !t->d_dist ||
        !t->d_pqk || !t->d_pqh || !t->d_pqs || !t->d_pqn)
        return give_up("device allocation", hipErrorOutOfMemory);
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&t->h_stage), 4 * (size_t(n) + 1) * dd, hipHostMallocDefault);
    if (e != hipSuccess) {
        t->h_stage = nullptr;
        return give_up("pinned staging allocation", e);
    }
    t->d_q = t->d_pts + size_t(n) * dd;
    if ((e = hipMemset(t->d_cd, 0xff, 4 * size_t(t->cap))) != hipSuccess) return give_up("hipMemset", e);
    if (n > 0) {
        stage_points(t, nullptr, fn);
        if ((e = gsc_launch_ann_build(t->d_pts, n, dd, t->d_pidx, t->d_cd, t->d_cv, t->d_lo, t->d_hi, t->d_bnd,
                                      t->d_dist, nullptr)) != hipSuccess)
            return give_up("tree build launch", e);
        if ((e = hipDeviceSynchronize()) != hipSuccess) return give_up("tree build", e);
    }
    return t;
}

void ann_kdtree_destroy(ann_kdtree_t* t) {
    if (!t) return;
    t->release();
    delete t;
}

static void ann_query(ann_kdtree_t* t, int* idxs, float* errs, int cnt, const float* q, float eps, int mode,
                      const char* fn) {
    if (!t) fatal(fn, "null tree (ann_kdtree_create failed)");
    if (cnt <= 0) return;
    if (cnt > t->kcap) {  // grow the result buffers; kcap changes only on success
        int* ni = dalloc<int>(size_t(cnt));
        float* ne = dalloc<float>(size_t(cnt));
        float* nm = dalloc<float>(size_t(cnt) + 1);
        int* nmi = dalloc<int>(size_t(cnt) + 1);
        int* ho = nullptr;
        if (hipHostMalloc(reinterpret_cast<void**>(&ho), 8 * size_t(cnt), hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            ho = nullptr;
        }
        if (!ni || !ne || !nm || !nmi || !ho) {
            dfree(ni);
            dfree(ne);
            dfree(nm);
            dfree(nmi);
            if (ho) (void)hipHostFree(ho);
            fatal(fn, "device allocation failed");
        }
        dfree(t->d_idx);
        dfree(t->d_err);
        dfree(t->d_mk);
        dfree(t->d_mki);
        if (t->h_out) (void)hipHostFree(t->h_out);
        t->d_idx = ni;
        t->d_err = ne;
        t->d_mk = nm;
        t->d_mki = nmi;
        t->h_out = ho;
        t->kcap = cnt;
    }
    if (t->n > 0) stage_points(t, q, fn);  // live values (the tree itself stays stale)
    check(fn, gsc_launch_ann_query(t->d_pts, t->n, t->dd, t->d_pidx, t->d_cd, t->d_cv, t->d_lo, t->d_hi, t->d_bnd,
                                   t->d_q, cnt, mode, eps, t->d_idx, t->d_err, t->d_dist, t->d_mk, t->d_mki, t->d_pqk,
                                   t->d_pqh, t->d_pqs, t->d_pqn, nullptr));
    check(fn, hipMemcpy(t->h_out, t->d_idx, 4 * size_t(cnt), hipMemcpyDeviceToHost));
    check(fn, hipMemcpy(t->h_out + cnt, t->d_err, 4 * size_t(cnt), hipMemcpyDeviceToHost));
    std::memcpy(idxs, t->h_out, 4 * size_t(cnt));
    std::memcpy(errs, t->h_out + cnt, 4 * size_t(cnt));
}

int ann_kdtree_search(ann_kdtree_t* akd, float* q, float eps, float* err) {
    int idx = -1;
    float e = 0;
    ann_query(akd, &idx, &e, 1, q, eps, 0, "ann_kdtree_search");
    if (err) *err = e;
    return idx;
}

int ann_kdtree_pri_search(ann_kdtree_t* akd, float* q, float eps, float* err) {
    int idx = -1;
    float e = 0;
    ann_query(akd, &idx, &e, 1, q, eps, 1, "ann_kdtree_pri_search");
    if (err) *err = e;
    return idx;
}

void ann_kdtree_search_multi(ann_kdtree_t* akd, int* idxs, float* errs, int cnt, float* q, float eps) {
    ann_query(akd, idxs, errs, cnt, q, eps, 0, "ann_kdtree_search_multi");
}

void ann_kdtree_pri_search_multi(ann_kdtree_t* akd, int* idxs, float* errs, int cnt, float* q, float eps) {
    ann_query(akd, idxs, errs, cnt, q, eps, 1, "ann_kdtree_pri_search_multi");
}

}  // extern "C"
