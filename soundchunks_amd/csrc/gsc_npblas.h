// Summation orders of the numpy / scipy BLAS calls that cluster.py's
// sklearn.cluster.Birch makes, restated so the -py reducer
// reproduces cluster.py's labels bit for bit.  The pin is the BLAS the
// reference's cluster.py runs with in the build container: OpenBLAS 0.3.29
// (numpy 2.2 / scipy wheels, DYNAMIC_ARCH, core "SkylakeX") and numpy's
// einsum baseline (SSE2) loops.  Every order below was derived from the
// library's kernels and checked element for element against numpy / scipy on
// random inputs at d = 8, 16, 32 (tools/birch/blas_orders.py):
//   np_ddot     np.dot(v, v) and scipy's ddot (sklearn _dot): OpenBLAS
//               ddot_k SkylakeX -- four 8-lane fma accumulators over blocks
//               of 32, folded to four 4-lane accumulators, blocks of 16 with
//               those four, lane-wise ((a0 + a1) + a2) + a3, then
//               (l0 + l2) + (l1 + l3), then a sequential fma tail
//   np_gemv_row np.dot(M, v), M row-major m x d (dgemv_t_SKYLAKEX): rows in
//               groups of 4 use dgemv_kernel_4x4 (one 4-lane fma accumulator
//               per row, (l0 + l2) + (l1 + l3)); the m % 4 leftover rows use
//               the SSE kernels 4x2 (two lanes, unfused mul / add) and 4x1
//               (two 2-lane accumulators, unfused); m == 1 is numpy's ddot
//   np_einsum_sq np.einsum('ij,ij->i', X, X) (sklearn row_norms): two lanes,
//               blocks of 8 added last-pair-first, unfused, lane 0 + lane 1
//   np_syrk51   numpy X @ X.T on one buffer (cblas_dsyrk) for the 51 x d
//               node centroids of _split_node: sequential fma chains, except
//               the 4-accumulator ((a0 + a1) + (a2 + a3)) order of the
//               remainder tile (columns 48..50 of rows 0..23 and 32..43)
//   scipy dgemm (Birch._predict's middle term): sequential fma chain
#pragma once
#include <cmath>

#if defined(__HIPCC__)
#define GSC_HD __host__ __device__
#else
#define GSC_HD
#endif

namespace gsc {
namespace npblas {

GSC_HD inline double fmad(double a, double b, double c) { return std::fma(a, b, c); }

// OpenBLAS ddot (SkylakeX kernel), unit strides
GSC_HD inline double np_ddot(const double* x, const double* y, int n) {
    double z[4][8];
    for (int r = 0; r < 4; ++r)
        for (int l = 0; l < 8; ++l) z[r][l] = 0.0;
    const int n16 = n & -16;
    const int n32 = n & -32;
    int i = 0;
    for (; i < n32; i += 32)
        for (int r = 0; r < 4; ++r)
            for (int l = 0; l < 8; ++l) z[r][l] = fmad(x[i + 8 * r + l], y[i + 8 * r + l], z[r][l]);
    double a[4][4];
    for (int r = 0; r < 4; ++r)
        for (int l = 0; l < 4; ++l) a[r][l] = z[r][l] + z[r][l + 4];
    for (; i < n16; i += 16)
        for (int r = 0; r < 4; ++r)
            for (int l = 0; l < 4; ++l) a[r][l] = fmad(x[i + 4 * r + l], y[i + 4 * r + l], a[r][l]);
    double b[4];
    for (int l = 0; l < 4; ++l) b[l] = ((a[0][l] + a[1][l]) + a[2][l]) + a[3][l];
    double s = (b[0] + b[2]) + (b[1] + b[3]);
    for (; i < n; ++i) s = fmad(x[i], y[i], s);
    return s;
}

// element i of np.dot(M, v) for a row-major m x n matrix (n a multiple of 4)
inline double np_gemv_row(const double* row, const double* v, int n, int m, int i) {
    if (m == 1) return np_ddot(row, v, n);
    const int q = 4 * (m / 4);
    if (i < q) {  // dgemv_kernel_4x4
        double t[4] = {0.0, 0.0, 0.0, 0.0};
        for (int k = 0; k < n; k += 4)
            for (int l = 0; l < 4; ++l) t[l] = fmad(row[k + l], v[k + l], t[l]);
        return (t[0] + t[2]) + (t[1] + t[3]);
    }
    if (((m % 4) & 2) && i < q + 2) {  // dgemv_kernel_4x2 (SSE, unfused)
        double t[2] = {0.0, 0.0};
        int k = 0;
        if (n & 2) {
            for (int l = 0; l < 2; ++l) t[l] = t[l] + row[l] * v[l];
            k = 2;
        }
        for (; k < n; k += 2)
            for (int l = 0; l < 2; ++l) t[l] = t[l] + row[k + l] * v[k + l];
        return t[0] + t[1];
    }
    // dgemv_kernel_4x1 (SSE, unfused, two accumulators)
    double p[2] = {0.0, 0.0}, r[2] = {0.0, 0.0};
    int k = 0;
    if (n & 2) {
        for (int l = 0; l < 2; ++l) p[l] = p[l] + row[l] * v[l];
        k = 2;
    }
    for (; k < n; k += 4)
        for (int l = 0; l < 2; ++l) {
            p[l] = p[l] + row[k + l] * v[k + l];
            r[l] = r[l] + row[k + 2 + l] * v[k + 2 + l];
        }
    return (p[0] + r[0]) + (p[1] + r[1]);
}

// np.einsum('ij,ij->i', X, X) for one row (numpy's SSE2 sum-of-products loop)
GSC_HD inline double np_einsum_sq(const double* x, int n) {
    double a[2] = {0.0, 0.0};
    int c = n, o = 0;
    for (; c >= 8; c -= 8, o += 8)
        for (int j = 3; j >= 0; --j)
            for (int l = 0; l < 2; ++l) a[l] = a[l] + x[o + 2 * j + l] * x[o + 2 * j + l];
    for (; c > 0; c -= 2, o += 2)
        for (int l = 0; l < 2; ++l) {
            const double v = l < c ? x[o + l] : 0.0;
            a[l] = a[l] + v * v;
        }
    return 0.0 + (a[0] + a[1]);
}

// sequential fma chain (OpenBLAS dgemm element order at these shapes)
GSC_HD inline double seq_fma_dot(const double* x, const double* y, int n) {
    double s = 0.0;
    for (int k = 0; k < n; ++k) s = fmad(x[k], y[k], s);
    return s;
}

// element (i, j), i <= j, of numpy's C @ C.T for the 51-row node centroid
// matrix of _split_node (cblas_dsyrk, upper triangle, mirrored)
inline double np_syrk51(const double* C, int n, int i, int j) {
    if (i > j) {
        const int t = i;
        i = j;
        j = t;
    }
    const double* x = C + static_cast<long>(i) * n;
    const double* y = C + static_cast<long>(j) * n;
    if (j >= 48 && (i < 24 || (i >= 32 && i < 44))) {
        double t[4] = {0.0, 0.0, 0.0, 0.0};
        for (int k = 0; k < n; k += 4)
            for (int l = 0; l < 4; ++l) t[l] = fmad(x[k + l], y[k + l], t[l]);
        return (t[0] + t[1]) + (t[2] + t[3]);
    }
    return seq_fma_dot(x, y, n);
}

}  // namespace npblas
}  // namespace gsc
