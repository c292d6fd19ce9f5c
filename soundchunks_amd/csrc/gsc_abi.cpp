// The extern.pas:112-123 drop-in surface (yakmo_single.dll + ANN.dll exports)
// implemented on the GPU.  Semantics follow the DLLs as the reference uses
// them: yakmo copies its training rows; ANN keeps the caller's row pointers
// and every search reads the points' *current* values (KNNScanReduce relies on
// that, encoder.lpr:729-745), so each search re-uploads the live rows.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/soundchunks.h"
#include "gsc_device.h"

extern "C" hipError_t gsc_launch_yakmo(int D, const gsc::ReduceFrame* frames, int nframes, const float* X, float* C,
                                       float* fs, int* is, uint32_t* bits, hipStream_t st);
extern "C" hipError_t gsc_launch_ann_build(const float* pts, int n, int dd, int* pidx, int* cd, float* cv, float* lo,
                                           float* hi, float* bnd, hipStream_t st);
extern "C" hipError_t gsc_launch_ann_query(const float* pts, int n, int dd, int* pidx, int* cd, float* cv, float* lo,
                                           float* hi, float* bnd, const float* q, int k, int mode, float eps,
                                           int* idxs, float* errs, float* mk_key, int* mk_info, float* pq_key,
                                           int* pq_h, int* pq_s, int* pq_n, hipStream_t st);

namespace {

void abi_error(const char* fn, const char* what) { std::fprintf(stderr, "soundchunks_amd: %s: %s\n", fn, what); }

#define ABI_HIP(fn, expr)                                  \
    do {                                                   \
        hipError_t e_ = (expr);                            \
        if (e_ != hipSuccess) {                            \
            abi_error(fn, hipGetErrorString(e_));          \
            return;                                        \
        }                                                  \
    } while (0)

template <typename T>
T* dalloc(size_t n) {
    T* p = nullptr;
    if (hipMalloc(&p, sizeof(T) * (n ? n : 1)) != hipSuccess) return nullptr;
    return p;
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
    int* d_idx = nullptr;
    float* d_err = nullptr;
    float* d_mk = nullptr;
    int* d_mki = nullptr;
    float* d_pqk = nullptr;
    int *d_pqh = nullptr, *d_pqs = nullptr, *d_pqn = nullptr;
    int kcap = 0;
    std::vector<float> staging;
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
    if (!y->supported) abi_error("yakmo_create", "only yakmo_create(K,1,0,1,0,0,v) is implemented");
    return y;
}

void yakmo_destroy(yakmo_t* ay) { delete ay; }

void yakmo_load_train_data(yakmo_t* ay, unsigned int rowCount, unsigned int colCount, float** dataset) {
    ay->rows = rowCount;
    ay->cols = colCount;
    ay->data.resize(size_t(rowCount) * colCount);
    for (unsigned r = 0; r < rowCount; ++r) std::memcpy(&ay->data[size_t(r) * colCount], dataset[r], 4 * colCount);
}

void yakmo_train_on_data(yakmo_t* ay, int* pointToCluster) {
    const int N = int(ay->rows), D = int(ay->cols), K = int(ay->k);
    if (!ay->supported || K <= 0 || K >= N || N > 262144 || !(D == 8 || D == 16 || D == 32)) {
        abi_error("yakmo_train_on_data", "unsupported configuration");
        return;
    }
    gsc::ReduceFrame fr{};
    fr.N = N;
    fr.K = K;
    fr.k_off = N;
    float *dX = dalloc<float>(ay->data.size()), *dC = dalloc<float>(size_t(K) * D), *dF = dalloc<float>(4 * size_t(N));
    int* dI = dalloc<int>(size_t(N) + K);
    uint32_t* dB = dalloc<uint32_t>(size_t(N) / 32 + 4);
    gsc::ReduceFrame* dFr = dalloc<gsc::ReduceFrame>(1);
    ABI_HIP("yakmo_train_on_data", hipMemcpy(dX, ay->data.data(), 4 * ay->data.size(), hipMemcpyHostToDevice));
    ABI_HIP("yakmo_train_on_data", hipMemcpy(dFr, &fr, sizeof(fr), hipMemcpyHostToDevice));
    ABI_HIP("yakmo_train_on_data", gsc_launch_yakmo(D, dFr, 1, dX, dC, dF, dI, dB, nullptr));
    ay->centroids.resize(size_t(K) * D);
    ay->labels.resize(size_t(N));
    ABI_HIP("yakmo_train_on_data", hipMemcpy(ay->centroids.data(), dC, 4 * ay->centroids.size(), hipMemcpyDeviceToHost));
    ABI_HIP("yakmo_train_on_data", hipMemcpy(ay->labels.data(), dI, 4 * size_t(N), hipMemcpyDeviceToHost));
    if (pointToCluster) std::memcpy(pointToCluster, ay->labels.data(), 4 * size_t(N));
    (void)hipFree(dX);
    (void)hipFree(dC);
    (void)hipFree(dF);
    (void)hipFree(dI);
    (void)hipFree(dB);
    (void)hipFree(dFr);
}

void yakmo_get_centroids(yakmo_t* ay, float** centroids) {
    for (unsigned c = 0; c < ay->k && (size_t(c) + 1) * ay->cols <= ay->centroids.size(); ++c)
        std::memcpy(centroids[c], &ay->centroids[size_t(c) * ay->cols], 4 * ay->cols);
}

// ---- ANN.dll -----------------------------------------------------------------
static bool upload_points(ann_kdtree_t* t) {
    for (int i = 0; i < t->n; ++i) std::memcpy(&t->staging[size_t(i) * t->dd], t->pa[i], 4 * size_t(t->dd));
    return hipMemcpy(t->d_pts, t->staging.data(), 4 * t->staging.size(), hipMemcpyHostToDevice) == hipSuccess;
}

ann_kdtree_t* ann_kdtree_create(float** pa, int n, int dd, int bs, int split) {
    if (bs != 1 || split != 0) {
        abi_error("ann_kdtree_create", "only bs = 1, ANN_KD_STD is implemented");
        return nullptr;
    }
    ann_kdtree_t* t = new ann_kdtree_t();
    t->pa = pa;
    t->n = n;
    t->dd = dd;
    int p2 = 1;
    while (p2 < (n > 0 ? n : 1)) p2 <<= 1;
    t->cap = 2 * p2;
    t->staging.resize(size_t(n) * dd);
    t->d_pts = dalloc<float>(size_t(n) * dd);
    t->d_pidx = dalloc<int>(size_t(n));
    t->d_cd = dalloc<int>(size_t(t->cap));
    t->d_cv = dalloc<float>(size_t(t->cap));
    t->d_lo = dalloc<float>(size_t(t->cap));
    t->d_hi = dalloc<float>(size_t(t->cap));
    t->d_bnd = dalloc<float>(2 * size_t(dd));
    t->d_q = dalloc<float>(size_t(dd));
    t->d_pqk = dalloc<float>(size_t(n) + 2);
    t->d_pqh = dalloc<int>(size_t(n) + 2);
    t->d_pqs = dalloc<int>(size_t(n) + 2);
    t->d_pqn = dalloc<int>(size_t(n) + 2);
    if (!t->d_pts || !t->d_pidx || !t->d_pqn) {
        abi_error("ann_kdtree_create", "device allocation failed");
        delete t;
        return nullptr;
    }
    (void)hipMemset(t->d_cd, 0xff, 4 * size_t(t->cap));
    if (n > 0) {
        if (!upload_points(t) ||
            gsc_launch_ann_build(t->d_pts, n, dd, t->d_pidx, t->d_cd, t->d_cv, t->d_lo, t->d_hi, t->d_bnd, nullptr) !=
                hipSuccess) {
            abi_error("ann_kdtree_create", "tree build failed");
        }
    }
    return t;
}

void ann_kdtree_destroy(ann_kdtree_t* t) {
    if (!t) return;
    for (void* p : {(void*)t->d_pts, (void*)t->d_pidx, (void*)t->d_cd, (void*)t->d_cv, (void*)t->d_lo, (void*)t->d_hi,
                    (void*)t->d_bnd, (void*)t->d_q, (void*)t->d_idx, (void*)t->d_err, (void*)t->d_mk, (void*)t->d_mki,
                    (void*)t->d_pqk, (void*)t->d_pqh, (void*)t->d_pqs, (void*)t->d_pqn})
        if (p) (void)hipFree(p);
    delete t;
}

static void ann_query(ann_kdtree_t* t, int* idxs, float* errs, int cnt, const float* q, float eps, int mode) {
    if (cnt > t->kcap) {
        for (void* p : {(void*)t->d_idx, (void*)t->d_err, (void*)t->d_mk, (void*)t->d_mki})
            if (p) (void)hipFree(p);
        t->kcap = cnt;
        t->d_idx = dalloc<int>(size_t(cnt));
        t->d_err = dalloc<float>(size_t(cnt));
        t->d_mk = dalloc<float>(size_t(cnt) + 1);
        t->d_mki = dalloc<int>(size_t(cnt) + 1);
    }
    if (!upload_points(t)) {  // live values (the tree itself stays stale)
        abi_error("ann_kdtree_search", "point upload failed");
        return;
    }
    ABI_HIP("ann_kdtree_search", hipMemcpy(t->d_q, q, 4 * size_t(t->dd), hipMemcpyHostToDevice));
    ABI_HIP("ann_kdtree_search",
            gsc_launch_ann_query(t->d_pts, t->n, t->dd, t->d_pidx, t->d_cd, t->d_cv, t->d_lo, t->d_hi, t->d_bnd,
                                 t->d_q, cnt, mode, eps, t->d_idx, t->d_err, t->d_mk, t->d_mki, t->d_pqk, t->d_pqh,
                                 t->d_pqs, t->d_pqn, nullptr));
    ABI_HIP("ann_kdtree_search", hipMemcpy(idxs, t->d_idx, 4 * size_t(cnt), hipMemcpyDeviceToHost));
    ABI_HIP("ann_kdtree_search", hipMemcpy(errs, t->d_err, 4 * size_t(cnt), hipMemcpyDeviceToHost));
}

int ann_kdtree_search(ann_kdtree_t* akd, float* q, float eps, float* err) {
    int idx = -1;
    float e = 0;
    ann_query(akd, &idx, &e, 1, q, eps, 0);
    if (err) *err = e;
    return idx;
}

int ann_kdtree_pri_search(ann_kdtree_t* akd, float* q, float eps, float* err) {
    int idx = -1;
    float e = 0;
    ann_query(akd, &idx, &e, 1, q, eps, 1);
    if (err) *err = e;
    return idx;
}

void ann_kdtree_search_multi(ann_kdtree_t* akd, int* idxs, float* errs, int cnt, float* q, float eps) {
    ann_query(akd, idxs, errs, cnt, q, eps, 0);
}

void ann_kdtree_pri_search_multi(ann_kdtree_t* akd, int* idxs, float* errs, int cnt, float* q, float eps) {
    ann_query(akd, idxs, errs, cnt, q, eps, 1);
}

}  // extern "C"
