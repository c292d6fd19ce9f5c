// FPC 3.2.2 RTL sin/cos/ln restated for the product runtime (see fpc_math.h).
// Compiled with -ffp-contract=off: the reference code has no FMA.
#include "fpc_math.h"

#include <cmath>
#include <cstring>

namespace gsc {
namespace fpc {
namespace {

inline uint32_t hi32(double x) { uint64_t u; std::memcpy(&u, &x, 8); return uint32_t(u >> 32); }
inline uint32_t lo32(double x) { uint64_t u; std::memcpy(&u, &x, 8); return uint32_t(u); }
inline double with_hi32(double x, uint32_t h) {
    uint64_t u; std::memcpy(&u, &x, 8);
    u = (u & 0xffffffffull) | (uint64_t(h) << 32);
    std::memcpy(&x, &u, 8);
    return x;
}

// 2/pi in base 2^24 (fdlibm ipio2); identical to the table in encoder.exe
constexpr int32_t kTwoOverPi[66] = {
    0xA2F983, 0x6E4E44, 0x1529FC, 0x2757D1, 0xF534DD, 0xC0DB62, 0x95993C, 0x439041, 0xFE5163, 0xABDEBB, 0xC561B7,
    0x246E3A, 0x424DD2, 0xE00649, 0x2EEA09, 0xD1921C, 0xFE1DEB, 0x1CB129, 0xA73EE8, 0x8235F5, 0x2EBB44, 0x84E99C,
    0x7026B4, 0x5F7E41, 0x3991D6, 0x398353, 0x39F49C, 0x845F8B, 0xBDF928, 0x3B1FF8, 0x97FFDE, 0x05980F, 0xEF2F11,
    0x8B5A0A, 0x6D1F6D, 0x367ECF, 0x27CB09, 0xB74F46, 0x3F669E, 0x5FEA2D, 0x7527BA, 0xC7EBE5, 0xF17B3D, 0x0739F7,
    0x8A5292, 0xEA6BFB, 0x5FB11F, 0x8D5D08, 0x560330, 0x46FC7B, 0x6BABF0, 0xCFBC20, 0x9AF436, 0x1DA9E3, 0x91615E,
    0xE61B08, 0x659985, 0x5F14A0, 0x68408D, 0xFFD880, 0x4D7327, 0x310606, 0x1556CA, 0x73A8C9, 0x60E27B, 0xC08C6B,
};
constexpr double kPio2Parts[8] = {
    1.57079625129699707031e+00, 7.54978941586159635335e-08, 5.39030252995776476554e-15, 3.28200341580791294123e-22,
    1.27065575308067607349e-29, 1.22933308981111328932e-36, 2.73370053816464559624e-44, 2.16741683877804819444e-51,
};

// fdlibm __kernel_rem_pio2, prec = 2 (jk = 4), as FPC calls it
int rem_pio2_large(const double* x, double* y, int e0, int nx) {
    constexpr double two24 = 16777216.0, twon24 = 5.96046447753906250000e-08;
    const int jk = 4, jp = 4;
    int iq[20];
    double f[20], fq[20], q[20];
    const int jx = nx - 1;
    int jv = (e0 - 3) / 24;
    if (jv < 0) jv = 0;
    int q0 = e0 - 24 * (jv + 1);
    for (int i = 0, j = jv - jx; i <= jx + jk; ++i, ++j) f[i] = j < 0 ? 0.0 : double(kTwoOverPi[j]);
    for (int i = 0; i <= jk; ++i) {
        double fw = 0.0;
        for (int j = 0; j <= jx; ++j) fw += x[j] * f[jx + i - j];
        q[i] = fw;
    }
    int jz = jk, n, ih;
    double z;
    for (;;) {
        z = q[jz];
        for (int i = 0, j = jz; j > 0; ++i, --j) {
            const double fw = double(int32_t(twon24 * z));
            iq[i] = int32_t(z - two24 * fw);
            z = q[j - 1] + fw;
        }
        z = std::ldexp(z, q0);
        z -= 8.0 * std::floor(z * 0.125);
        n = int32_t(z);
        z -= double(n);
        ih = 0;
        if (q0 > 0) {
            const int i = iq[jz - 1] >> (24 - q0);
            n += i;
            iq[jz - 1] -= i << (24 - q0);
            ih = iq[jz - 1] >> (23 - q0);
        } else if (q0 == 0) {
            ih = iq[jz - 1] >> 23;
        } else if (z >= 0.5) {
            ih = 2;
        }
        if (ih > 0) {
            n += 1;
            int carry = 0;
            for (int i = 0; i < jz; ++i) {
                const int j = iq[i];
                if (carry == 0) {
                    if (j != 0) { carry = 1; iq[i] = 0x1000000 - j; }
                } else {
                    iq[i] = 0xffffff - j;
                }
            }
            if (q0 == 1) iq[jz - 1] &= 0x7fffff;
            else if (q0 == 2) iq[jz - 1] &= 0x3fffff;
            if (ih == 2) {
                z = 1.0 - z;
                if (carry != 0) z -= std::ldexp(1.0, q0);
            }
        }
        if (z == 0.0) {
            int j = 0;
            for (int i = jz - 1; i >= jk; --i) j |= iq[i];
            if (j == 0) {
                int k = 1;
                while (iq[jk - k] == 0) ++k;
                for (int i = jz + 1; i <= jz + k; ++i) {
                    f[jx + i] = double(kTwoOverPi[jv + i]);
                    double fw = 0.0;
                    for (int jj = 0; jj <= jx; ++jj) fw += x[jj] * f[jx + i - jj];
                    q[i] = fw;
                }
                jz += k;
                continue;  // recompute
            }
        }
        break;
    }
    if (z == 0.0) {
        jz -= 1;
        q0 -= 24;
        while (iq[jz] == 0) { --jz; q0 -= 24; }
    } else {
        z = std::ldexp(z, -q0);
        if (z >= two24) {
            const double fw = double(int32_t(twon24 * z));
            iq[jz] = int32_t(z - two24 * fw);
            ++jz;
            q0 += 24;
            iq[jz] = int32_t(fw);
        } else {
            iq[jz] = int32_t(z);
        }
    }
    double fw = std::ldexp(1.0, q0);
    for (int i = jz; i >= 0; --i) { q[i] = fw * double(iq[i]); fw *= twon24; }
    for (int i = jz; i >= 0; --i) {
        double acc = 0.0;
        for (int k = 0; k <= jp && k <= jz - i; ++k) acc += kPio2Parts[k] * q[i + k];
        fq[jz - i] = acc;
    }
    double acc = 0.0;
    for (int i = jz; i >= 0; --i) acc += fq[i];
    y[0] = ih == 0 ? acc : -acc;
    acc = fq[0] - acc;
    for (int i = 1; i <= jz; ++i) acc += fq[i];
    y[1] = ih == 0 ? acc : -acc;
    return n & 7;
}

double floor_fpc(double x) {
    const double t = std::trunc(x);
    if (x >= 0.0 || t == x) return t;
    return t - 1.0;
}

// FPC rem_pio2: quadrant count mod 8 and remainder in [-pi/4, pi/4]
long rem_pio2(double x, double* y) {
    constexpr double kPio4 = 7.85398163397448309616e-1;
    constexpr double kDp1 = 7.85398125648498535156e-1, kDp2 = 3.77489470793079817668e-8,
                     kDp3 = 2.69515142907905952645e-15;
    const double ax = std::fabs(x);
    if (ax < kPio4) {
        *y = x;
        return 0;
    }
    if (ax < 1073741824.0) {
        double oct = floor_fpc(x / kPio4);
        const double hi = floor_fpc(oct * 0.0625) * 16.0;
        uint32_t j = uint32_t(int64_t(oct - hi));
        if (j & 1u) { ++j; oct += 1.0; }
        const double r = ((x - oct * kDp1) - oct * kDp2) - oct * kDp3;
        *y = r;
        if (std::fabs(r) > 2.384185791015625e-07) return long((j >> 1) & 7u);
    }
    double z = std::fabs(x);
    const uint32_t hx = hi32(z);
    const int e0 = int(hx >> 20) - 0x416;
    if (e0 == 0x3e9) {
        *y = x - x;
        return 0;
    }
    z = with_hi32(z, hx - (uint32_t(e0) << 20));
    double tx[3], ty[2];
    tx[0] = double(int64_t(z));
    z = (z - tx[0]) * 16777216.0;
    tx[1] = double(int64_t(z));
    z = (z - tx[1]) * 16777216.0;
    tx[2] = z;
    int nx = 3;
    while (tx[nx - 1] == 0.0) --nx;
    long n = rem_pio2_large(tx, ty, e0, nx);
    if (x < 0.0) {
        *y = -ty[0] - ty[1];
        return (-n) & 7;
    }
    *y = ty[0] + ty[1];
    return n;
}

constexpr double kSinCof[6] = {1.58962301576546568060E-10, -2.50507477628578072866E-8, 2.75573136213857245213E-6,
                               -1.98412698295895385996E-4, 8.33333333332211858878E-3,  -1.66666666666666307295E-1};
constexpr double kCosCof[6] = {-1.13585365213876817300E-11, 2.08757008419747316778E-9, -2.75573141792967388112E-7,
                               2.48015872888517045348E-5,   -1.38888888888730564116E-3, 4.16666666666665929218E-2};

inline double horner5(double x, const double* c) {
    double a = c[0];
    for (int i = 1; i < 6; ++i) a = a * x + c[i];
    return a;
}
inline double k_sin(double y) { return horner5(y * y, kSinCof) * ((y * y) * y) + y; }
inline double k_cos(double y) {
    const double zz = y * y;
    const double head = 1.0 - std::ldexp(zz, -1);
    return horner5(zz, kCosCof) * (zz * zz) + head;
}

}  // namespace

double sin(double x) {
    if (x == 0.0) return x;
    double y;
    const long q = rem_pio2(x, &y) & 3;
    double r = (q & 1) ? k_cos(y) : k_sin(y);
    return q > 1 ? -r : r;
}

double cos(double x) {
    double y;
    const long q = rem_pio2(x, &y) & 3;
    double r = (q & 1) ? k_sin(y) : k_cos(y);
    return (q == 1 || q == 2) ? -r : r;
}

int64_t round(double x) { return int64_t(std::nearbyint(x)); }

int64_t ceil_pos(double x) {
    const double t = std::trunc(x);
    int64_t r = int64_t(t);
    if (x - t > 0.0) ++r;
    return r;
}

}  // namespace fpc
}  // namespace gsc
