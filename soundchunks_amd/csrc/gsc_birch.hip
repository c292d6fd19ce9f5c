// Device parts of the -py (Birch) reducer (gsc_birch_host.cpp):
// the Ward linkage of the leaf subcluster centroids and Birch._predict.
//
// Ward linkage = scipy.cluster.hierarchy.ward (scipy 1.15): the condensed
// euclidean pdist (sequential f64 sum, sqrt), then the nearest-neighbour
// chain with the Lance-Williams Ward update, restated from scipy's
// _hierarchy.nn_chain (checked bit for bit against scipy on random, tied
// and duplicated inputs): the chain's top x scans every live cluster for its
// nearest neighbour, keeping the chain's previous element on a tie and the
// lowest index among equal minima; mutual neighbours merge into the higher
// index.  The scan and the distance update are parallel over clusters; the
// chain itself is sequential, so one workgroup runs the whole linkage.
// f64 arithmetic is the reference's (-ffp-contract=off: no FMA in the Ward
// update; sqrt and division correctly rounded).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <vector>

#include "gsc_npblas.h"

namespace gsc {
namespace {

constexpr int kWardThreads = 1024;

__device__ __forceinline__ int64_t cidx(int64_t n, int64_t i, int64_t j) {  // scipy condensed_index
    if (i > j) {
        const int64_t t = i;
        i = j;
        j = t;
    }
    return n * i - (i * (i + 1)) / 2 + (j - i - 1);
}

// scipy _hierarchy_distance_update.pxi: _ward
__device__ __forceinline__ double ward_update(double d_xi, double d_yi, double d_xy, int size_x, int size_y,
                                              int size_i) {
    const double t = 1.0 / (double)(size_x + size_y + size_i);
    return sqrt((double)(size_i + size_x) * t * d_xi * d_xi + (double)(size_i + size_y) * t * d_yi * d_yi -
                (double)size_i * t * d_xy * d_xy);
}

// scipy pdist 'euclidean': sqrt(sum_k (u_k - v_k)^2), sequential in k
__global__ __launch_bounds__(256) void pdist_kernel(int n, int d, const double* __restrict__ X, double* __restrict__ D) {
    const int64_t total = (int64_t)n * (n - 1) / 2;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
        // row i of the condensed layout: p < cidx(n, i, n-1) + 1
        int64_t i = (int64_t)((2.0 * n - 1.0 - sqrt((2.0 * n - 1.0) * (2.0 * n - 1.0) - 8.0 * (double)p)) / 2.0);
        if (i < 0) i = 0;
        while (i > 0 && cidx(n, i, i + 1) > p) --i;
        while (i + 2 <= n - 1 && cidx(n, i + 1, i + 2) <= p) ++i;
        const int64_t j = p - cidx(n, i, i + 1) + i + 1;
        const double* u = X + i * d;
        const double* v = X + j * d;
        double s = 0.0;
        for (int k = 0; k < d; ++k) {
            const double t = u[k] - v[k];
            s = s + t * t;
        }
        D[p] = sqrt(s);
    }
}

struct MinRec {
    double v;
    int i;
};
__device__ __forceinline__ MinRec minrec(MinRec a, MinRec b) {
    if (b.v < a.v || (b.v == a.v && b.i < a.i)) return b;
    return a;
}

// scipy _hierarchy.nn_chain (method = ward), one workgroup; Z rows
// (x, y, height, size) in merge order (the host sorts and relabels)
__global__ __launch_bounds__(kWardThreads) void ward_nn_chain_kernel(int n, double* __restrict__ D,
                                                                     int* __restrict__ size, int* __restrict__ chain,
                                                                     double* __restrict__ Z) {
    __shared__ MinRec part[kWardThreads / 64];
    __shared__ int s_x, s_y, s_cl, s_done;
    __shared__ double s_min;
    const int tid = threadIdx.x;
    for (int i = tid; i < n; i += kWardThreads) size[i] = 1;
    if (tid == 0) s_cl = 0;
    __syncthreads();
    for (int k = 0; k < n - 1; ++k) {
        if (s_cl == 0) {  // chain restarts at the first live cluster
            MinRec r{0.0, 0x7fffffff};
            for (int i = tid; i < n; i += kWardThreads)
                if (size[i] > 0 && i < r.i) r.i = i;
            for (int o = 32; o > 0; o >>= 1) r.i = min(r.i, __shfl_xor(r.i, o));
            if ((tid & 63) == 0) part[tid >> 6] = r;
            __syncthreads();
            if (tid == 0) {
                int f = 0x7fffffff;
                for (int w = 0; w < kWardThreads / 64; ++w) f = min(f, part[w].i);
                chain[0] = f;
                s_cl = 1;
            }
            __syncthreads();
        }
        for (;;) {
            const int cl = s_cl;
            const int x = chain[cl - 1];
            MinRec r{INFINITY, 0x7fffffff};
            for (int i = tid; i < n; i += kWardThreads) {
                if (size[i] == 0 || i == x) continue;
                r = minrec(r, MinRec{D[cidx(n, x, i)], i});
            }
            for (int o = 32; o > 0; o >>= 1) {
                MinRec q;
                q.v = __shfl_xor(r.v, o);
                q.i = __shfl_xor(r.i, o);
                r = minrec(r, q);
            }
            if ((tid & 63) == 0) part[tid >> 6] = r;
            __syncthreads();
            if (tid == 0) {
                MinRec g = part[0];
                for (int w = 1; w < kWardThreads / 64; ++w) g = minrec(g, part[w]);
                // the previous chain element wins ties (scipy starts from it
                // and only replaces it by a strictly smaller distance)
                int y;
                double cur;
                if (cl > 1) {
                    const int prev = chain[cl - 2];
                    const double dp = D[cidx(n, x, prev)];
                    if (g.v < dp) {
                        y = g.i;
                        cur = g.v;
                    } else {
                        y = prev;
                        cur = dp;
                    }
                } else {
                    y = g.i;
                    cur = g.v;
                }
                s_x = x;
                s_y = y;
                s_min = cur;
                if (cl > 1 && y == chain[cl - 2]) {
                    s_done = 1;
                } else {
                    chain[cl] = y;
                    s_cl = cl + 1;
                    s_done = 0;
                }
            }
            __syncthreads();
            if (s_done) break;
        }
        int x = s_x, y = s_y;
        const double cur = s_min;
        if (x > y) {
            const int t = x;
            x = y;
            y = t;
        }
        const int nx = size[x], ny = size[y];
        __syncthreads();  // every thread has read the sizes
        if (tid == 0) {
            Z[(int64_t)k * 4 + 0] = (double)x;
            Z[(int64_t)k * 4 + 1] = (double)y;
            Z[(int64_t)k * 4 + 2] = cur;
            Z[(int64_t)k * 4 + 3] = (double)(nx + ny);
            size[x] = 0;
            size[y] = nx + ny;
            s_cl = s_cl - 2;
        }
        __syncthreads();
        for (int i = tid; i < n; i += kWardThreads) {
            const int ni = size[i];
            if (ni == 0 || i == y) continue;
            D[cidx(n, i, y)] = ward_update(D[cidx(n, i, x)], D[cidx(n, i, y)], cur, nx, ny, ni);
        }
        __threadfence_block();
        __syncthreads();
    }
}

// Birch._predict = sklearn ArgKmin (k = 1) over EuclideanArgKmin64:
// d = max(0, (|x|^2 + (-2 x.c)) + |c|^2) with |x|^2 from scipy's ddot
// (_sqeuclidean_row_norms64), the middle term from scipy's dgemm (alpha = -2,
// a sequential fma chain per element) and |c|^2 = Birch._subcluster_norms
// (row_norms: einsum); heap_push keeps the first strict minimum.  One thread
// per sample.
__global__ __launch_bounds__(256) void birch_predict_kernel(int n, int d, const double* __restrict__ X, int m,
                                                            const double* __restrict__ C,
                                                            const double* __restrict__ cn,
                                                            int* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* x = X + (int64_t)i * d;
    const double xn = npblas::np_ddot(x, x, d);
    double best = INFINITY;
    int bi = 0;
    for (int j = 0; j < m; ++j) {
        const double mid = -2.0 * npblas::seq_fma_dot(x, C + (int64_t)j * d, d);
        double v = xn + mid;
        v = v + cn[j];
        v = v > 0.0 ? v : 0.0;  // max(0., d): catastrophic cancellation
        if (v < best) {
            best = v;
            bi = j;
        }
    }
    out[i] = bi;
}

__global__ void row_norms_kernel(int m, int d, const double* __restrict__ C, double* __restrict__ cn) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) cn[j] = npblas::np_einsum_sq(C + (int64_t)j * d, d);
}

template <typename T>
struct DBuf {
    T* p = nullptr;
    ~DBuf() {
        if (p) (void)hipFree(p);
    }
    bool alloc(size_t n) { return hipMalloc(&p, sizeof(T) * (n ? n : 1)) == hipSuccess; }
};

}  // namespace

// Ward linkage of m centroids (m x d, row major): Z[(m-1) x 4] in merge
// order (scipy's nn_chain output before its stable sort and relabelling)
extern "C" int gsc_ward_linkage_dev(int m, int d, const double* centers, double* Z) {
    if (m < 2) return 0;
    const int64_t nd = (int64_t)m * (m - 1) / 2;
    {  // the condensed distance matrix must fit: refuse up front (-2) instead of failing mid-way
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return -1;
        if ((size_t)nd * sizeof(double) + (size_t)m * (size_t)(d + 8) * sizeof(double) > free_b) return -2;
    }
    DBuf<double> dX, dD, dZ;
    DBuf<int> dS, dC;
    if (!dX.alloc(size_t(m) * d) || !dD.alloc(size_t(nd)) || !dZ.alloc(size_t(m - 1) * 4) || !dS.alloc(size_t(m)) ||
        !dC.alloc(size_t(m)))
        return -1;
    if (hipMemcpy(dX.p, centers, sizeof(double) * size_t(m) * d, hipMemcpyHostToDevice) != hipSuccess) return -1;
    const int64_t blocks = (nd + 255) / 256;
    hipLaunchKernelGGL(pdist_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, nullptr, m, d,
                       dX.p, dD.p);
    hipLaunchKernelGGL(ward_nn_chain_kernel, dim3(1), dim3(kWardThreads), 0, nullptr, m, dD.p, dS.p, dC.p, dZ.p);
    if (hipGetLastError() != hipSuccess) return -1;
    if (hipMemcpy(Z, dZ.p, sizeof(double) * size_t(m - 1) * 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return 0;
}

// nearest centroid (first minimum) of every sample
extern "C" int gsc_birch_predict_dev(int n, int d, const double* X, int m, const double* centers, int* argmin) {
    if (n <= 0) return 0;
    DBuf<double> dX, dC, dN;
    DBuf<int> dO;
    if (!dX.alloc(size_t(n) * d) || !dC.alloc(size_t(m) * d) || !dN.alloc(size_t(m)) || !dO.alloc(size_t(n)))
        return -1;
    if (hipMemcpy(dX.p, X, sizeof(double) * size_t(n) * d, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dC.p, centers, sizeof(double) * size_t(m) * d, hipMemcpyHostToDevice) != hipSuccess)
        return -1;
    hipLaunchKernelGGL(row_norms_kernel, dim3((m + 255) / 256), dim3(256), 0, nullptr, m, d, dC.p, dN.p);
    hipLaunchKernelGGL(birch_predict_kernel, dim3((n + 255) / 256), dim3(256), 0, nullptr, n, d, dX.p, m, dC.p, dN.p,
                       dO.p);
    if (hipGetLastError() != hipSuccess) return -1;
    if (hipMemcpy(argmin, dO.p, sizeof(int) * size_t(n), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return 0;
}

}  // namespace gsc
