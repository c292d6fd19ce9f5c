// CPU harness (development aid, not the product): gsc_birch_host.cpp's Birch with
// host restatements of the two device steps, to compare labels with the
// cluster.py fixtures on a machine without a GPU.
//   g++ -O2 -ffp-contract=off -shared -fPIC -o /tmp/birch_host.so tools/birch/host_check.cpp soundchunks_amd/csrc/gsc_birch_host.cpp
// (tests/test_birch_host.py builds and runs it against the cluster.py fixtures)
#include <cmath>
#include <string>
#include <vector>

#include "../../soundchunks_amd/csrc/gsc_npblas.h"

namespace gsc {
int birch_reduce_labels(int n, int d, const float* feat, int K, int* labels, std::string* err);

static long long cidx(long long n, long long i, long long j) {
    if (i > j) std::swap(i, j);
    return n * i - (i * (i + 1)) / 2 + (j - i - 1);
}
extern "C" int gsc_ward_linkage_dev(int n, int d, const double* X, double* Z) {
    std::vector<double> D(size_t((long long)n * (n - 1) / 2));
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j) {
            double s = 0.0;
            for (int k = 0; k < d; ++k) {
                const double t = X[size_t(i) * d + k] - X[size_t(j) * d + k];
                s = s + t * t;
            }
            D[size_t(cidx(n, i, j))] = std::sqrt(s);
        }
    std::vector<int> size(size_t(n), 1);
    std::vector<int> chain(static_cast<size_t>(n));
    int cl = 0;
    for (int k = 0; k < n - 1; ++k) {
        if (cl == 0) {
            cl = 1;
            for (int i = 0; i < n; ++i)
                if (size[i] > 0) {
                    chain[0] = i;
                    break;
                }
        }
        int x, y = 0;
        double cur;
        for (;;) {
            x = chain[cl - 1];
            if (cl > 1) {
                y = chain[cl - 2];
                cur = D[size_t(cidx(n, x, y))];
            } else {
                cur = INFINITY;
            }
            for (int i = 0; i < n; ++i) {
                if (size[i] == 0 || x == i) continue;
                const double dd = D[size_t(cidx(n, x, i))];
                if (dd < cur) {
                    cur = dd;
                    y = i;
                }
            }
            if (cl > 1 && y == chain[cl - 2]) break;
            chain[cl++] = y;
        }
        cl -= 2;
        if (x > y) std::swap(x, y);
        const int nx = size[x], ny = size[y];
        Z[size_t(k) * 4] = x;
        Z[size_t(k) * 4 + 1] = y;
        Z[size_t(k) * 4 + 2] = cur;
        Z[size_t(k) * 4 + 3] = nx + ny;
        size[x] = 0;
        size[y] = nx + ny;
        for (int i = 0; i < n; ++i) {
            const int ni = size[i];
            if (ni == 0 || i == y) continue;
            const double t = 1.0 / double(nx + ny + ni);
            const double dxi = D[size_t(cidx(n, i, x))], dyi = D[size_t(cidx(n, i, y))];
            D[size_t(cidx(n, i, y))] =
                std::sqrt(double(ni + nx) * t * dxi * dxi + double(ni + ny) * t * dyi * dyi - double(ni) * t * cur * cur);
        }
    }
    return 0;
}
// Birch._predict on the host (gsc_birch.hip birch_predict_kernel restated)
extern "C" int gsc_birch_predict_dev(int n, int d, const double* X, int m, const double* C, int* out) {
    std::vector<double> cn(static_cast<size_t>(m));
    for (int j = 0; j < m; ++j) cn[j] = npblas::np_einsum_sq(C + size_t(j) * d, d);
    for (int i = 0; i < n; ++i) {
        const double* x = X + size_t(i) * d;
        const double xn = npblas::np_ddot(x, x, d);
        double best = INFINITY;
        int bi = 0;
        for (int j = 0; j < m; ++j) {
            double v = xn + -2.0 * npblas::seq_fma_dot(x, C + size_t(j) * d, d);
            v = v + cn[j];
            v = v > 0.0 ? v : 0.0;
            if (v < best) {
                best = v;
                bi = j;
            }
        }
        out[i] = bi;
    }
    return 0;
}
}  // namespace gsc

extern "C" int birch_host_labels(int n, int d, const float* x, int k, int* labels) {
    std::string err;
    return gsc::birch_reduce_labels(n, d, x, k, labels, &err);
}
