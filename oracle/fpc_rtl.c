/*
 * ORACLE (test infrastructure only) -- FPC 3.2.2 Win64 RTL numerics restated.
 * See fpc_rtl.h for the disassembly anchors.  Compile with -ffp-contract=off:
 * the reference is plain SSE2 scalar code (no FMA anywhere).
 */
#include "fpc_rtl.h"

#include <math.h>
#include <stdint.h>
#include <string.h>

static inline uint32_t hi_word(double x) { uint64_t u; memcpy(&u, &x, 8); return (uint32_t)(u >> 32); }
static inline uint32_t lo_word(double x) { uint64_t u; memcpy(&u, &x, 8); return (uint32_t)u; }
static inline double set_hi_word(double x, uint32_t hi) {
    uint64_t u; memcpy(&u, &x, 8);
    u = (u & 0xffffffffull) | ((uint64_t)hi << 32);
    memcpy(&x, &u, 8);
    return x;
}

/* ---- fdlibm __kernel_rem_pio2 (encoder.exe @0x10000a500) ---------------- */
/* base-2^24 digits of 2/pi; verified against mpmath in tests */
static const int32_t two_over_pi[66] = {
    0xA2F983, 0x6E4E44, 0x1529FC, 0x2757D1, 0xF534DD, 0xC0DB62, 0x95993C, 0x439041, 0xFE5163,
    0xABDEBB, 0xC561B7, 0x246E3A, 0x424DD2, 0xE00649, 0x2EEA09, 0xD1921C, 0xFE1DEB, 0x1CB129,
    0xA73EE8, 0x8235F5, 0x2EBB44, 0x84E99C, 0x7026B4, 0x5F7E41, 0x3991D6, 0x398353, 0x39F49C,
    0x845F8B, 0xBDF928, 0x3B1FF8, 0x97FFDE, 0x05980F, 0xEF2F11, 0x8B5A0A, 0x6D1F6D, 0x367ECF,
    0x27CB09, 0xB74F46, 0x3F669E, 0x5FEA2D, 0x7527BA, 0xC7EBE5, 0xF17B3D, 0x0739F7, 0x8A5292,
    0xEA6BFB, 0x5FB11F, 0x8D5D08, 0x560330, 0x46FC7B, 0x6BABF0, 0xCFBC20, 0x9AF436, 0x1DA9E3,
    0x91615E, 0xE61B08, 0x659985, 0x5F14A0, 0x68408D, 0xFFD880, 0x4D7327, 0x310606, 0x1556CA,
    0x73A8C9, 0x60E27B, 0xC08C6B,
};
/* encoder.exe VA 0x10004b640 */
static const double PIo2[8] = {
    1.57079625129699707031e+00, 7.54978941586159635335e-08, 5.39030252995776476554e-15,
    3.28200341580791294123e-22, 1.27065575308067607349e-29, 1.22933308981111328932e-36,
    2.73370053816464559624e-44, 2.16741683877804819444e-51,
};
static const int init_jk[4] = {2, 3, 4, 6};

static int kernel_rem_pio2(const double *x, double *y, int e0, int nx, int prec) {
    const double two24 = 1.67772160000000000000e+07, twon24 = 5.96046447753906250000e-08;
    int jz, jx, jv, jp, jk, carry, n, iq[20], i, j, k, m, q0, ih;
    double z, fw, f[20], fq[20], q[20];

    jk = init_jk[prec];
    jp = jk;
    jx = nx - 1;
    jv = (e0 - 3) / 24;
    if (jv < 0) jv = 0;
    q0 = e0 - 24 * (jv + 1);
    j = jv - jx;
    m = jx + jk;
    for (i = 0; i <= m; i++, j++) f[i] = (j < 0) ? 0.0 : (double)two_over_pi[j];
    for (i = 0; i <= jk; i++) {
        for (j = 0, fw = 0.0; j <= jx; j++) fw += x[j] * f[jx + i - j];
        q[i] = fw;
    }
    jz = jk;
recompute:
    for (i = 0, j = jz, z = q[jz]; j > 0; i++, j--) {
        fw = (double)((int32_t)(twon24 * z));
        iq[i] = (int32_t)(z - two24 * fw);
        z = q[j - 1] + fw;
    }
    z = ldexp(z, q0);
    z -= 8.0 * floor(z * 0.125);
    n = (int32_t)z;
    z -= (double)n;
    ih = 0;
    if (q0 > 0) {
        i = (iq[jz - 1] >> (24 - q0));
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
        carry = 0;
        for (i = 0; i < jz; i++) {
            j = iq[i];
            if (carry == 0) {
                if (j != 0) { carry = 1; iq[i] = 0x1000000 - j; }
            } else {
                iq[i] = 0xffffff - j;
            }
        }
        if (q0 > 0) {
            switch (q0) {
            case 1: iq[jz - 1] &= 0x7fffff; break;
            case 2: iq[jz - 1] &= 0x3fffff; break;
            }
        }
        if (ih == 2) {
            z = 1.0 - z;
            if (carry != 0) z -= ldexp(1.0, q0);
        }
    }
    if (z == 0.0) {
        j = 0;
        for (i = jz - 1; i >= jk; i--) j |= iq[i];
        if (j == 0) {
            for (k = 1; iq[jk - k] == 0; k++) {}
            for (i = jz + 1; i <= jz + k; i++) {
                f[jx + i] = (double)two_over_pi[jv + i];
                for (j = 0, fw = 0.0; j <= jx; j++) fw += x[j] * f[jx + i - j];
                q[i] = fw;
            }
            jz += k;
            goto recompute;
        }
    }
    if (z == 0.0) {
        jz -= 1;
        q0 -= 24;
        while (iq[jz] == 0) { jz--; q0 -= 24; }
    } else {
        z = ldexp(z, -q0);
        if (z >= two24) {
            fw = (double)((int32_t)(twon24 * z));
            iq[jz] = (int32_t)(z - two24 * fw);
            jz += 1;
            q0 += 24;
            iq[jz] = (int32_t)fw;
        } else {
            iq[jz] = (int32_t)z;
        }
    }
    fw = ldexp(1.0, q0);
    for (i = jz; i >= 0; i--) { q[i] = fw * (double)iq[i]; fw *= twon24; }
    for (i = jz; i >= 0; i--) {
        for (fw = 0.0, k = 0; k <= jp && k <= jz - i; k++) fw += PIo2[k] * q[i + k];
        fq[jz - i] = fw;
    }
    /* prec == 2 (the only caller's value) */
    fw = 0.0;
    for (i = jz; i >= 0; i--) fw += fq[i];
    y[0] = (ih == 0) ? fw : -fw;
    fw = fq[0] - fw;
    for (i = 1; i <= jz; i++) fw += fq[i];
    y[1] = (ih == 0) ? fw : -fw;
    return n & 7;
}

/* ---- FPC floor (encoder.exe @0x10000a4b0) ------------------------------- */
static double fpc_floor(double x) {
    double t = trunc(x);
    if (x >= 0.0) return t;
    if (t == x) return t;
    return t - 1.0;
}

/* ---- rem_pio2 (encoder.exe @0x10000b150) -------------------------------- */
long fpc_rem_pio2(double x, double *y) {
    const double PIO4 = 7.85398163397448309616e-1;
    const double DP1 = 7.85398125648498535156e-1;
    const double DP2 = 3.77489470793079817668e-8;
    const double DP3 = 2.69515142907905952645e-15;
    const double TOL = 2.384185791015625e-07; /* 2^-22, VA 0x10004b7c0 */
    double ax = fabs(x);
    long n;
    if (ax < PIO4) { /* jp/jae: NaN falls through to the >= path */
        *y = x;
        return 0;
    }
    if (ax < 1073741824.0) {
        double yy = fpc_floor(x / PIO4);
        double z = fpc_floor(yy * 0.0625) * 16.0;
        int64_t jj = (int64_t)(yy - z);
        uint32_t j = (uint32_t)jj;
        if (j & 1) { j += 1; yy += 1.0; }
        double r = ((x - yy * DP1) - yy * DP2) - yy * DP3;
        *y = r;
        n = (long)((j >> 1) & 7);
        if (fabs(r) > TOL) return n;
        /* |r| <= 2^-22 (or NaN): fall into the precise path */
    }
    {
        double z = fabs(x);
        uint32_t hx = hi_word(z);
        int e0 = (int)(hx >> 20) - 0x416;
        if (e0 == 0x3e9) { /* inf / nan */
            *y = x - x;
            return 0;
        }
        z = set_hi_word(z, hx - ((uint32_t)e0 << 20));
        double tx[3], ty[2];
        tx[0] = (double)(int64_t)z;
        z = (z - tx[0]) * 16777216.0;
        tx[1] = (double)(int64_t)z;
        z = (z - tx[1]) * 16777216.0;
        tx[2] = z;
        int nx = 3;
        while (tx[nx - 1] == 0.0) nx--;
        n = kernel_rem_pio2(tx, ty, e0, nx, 2);
        if (x < 0.0) {
            n = (-n) & 7;
            *y = -ty[0] - ty[1];
        } else {
            *y = ty[0] + ty[1];
        }
        return n;
    }
}

/* ---- polevl (encoder.exe @0x10000a480): Horner, separate mul/add --------- */
static double polevl5(double x, const double *c) {
    double a = c[0];
    for (int i = 1; i <= 5; i++) a = a * x + c[i];
    return a;
}

static const double sincof[6] = {
    1.58962301576546568060E-10, -2.50507477628578072866E-8, 2.75573136213857245213E-6,
    -1.98412698295895385996E-4, 8.33333333332211858878E-3,  -1.66666666666666307295E-1,
};
static const double coscof[6] = {
    -1.13585365213876817300E-11, 2.08757008419747316778E-9, -2.75573141792967388112E-7,
    2.48015872888517045348E-5,   -1.38888888888730564116E-3, 4.16666666666665929218E-2,
};

static inline double sin_kernel(double y) { /* poly*(y*y*y) + y */
    double zz = y * y;
    double p = polevl5(zz, sincof);
    double y3 = (y * y) * y;
    return p * y3 + y;
}
static inline double cos_kernel(double y) { /* poly*zz^2 + (1 - zz/2) */
    double zz = y * y;
    double h = 1.0 - ldexp(zz, -1);
    double zz2 = zz * zz;
    return polevl5(zz, coscof) * zz2 + h;
}

double fpc_sin(double x) {
    if (x == 0.0) return x;
    double y;
    long n = fpc_rem_pio2(x, &y) & 3;
    double r = (n == 1 || n == 3) ? cos_kernel(y) : sin_kernel(y);
    if (n > 1) r = -r;
    return r;
}

double fpc_cos(double x) {
    double y;
    long n = fpc_rem_pio2(x, &y) & 3;
    double r = (n == 1 || n == 3) ? sin_kernel(y) : cos_kernel(y);
    if (n == 1 || n == 2) r = -r;
    return r;
}

/* ---- fdlibm __ieee754_log (encoder.exe @0x10000b690) --------------------- */
double fpc_ln(double x) {
    static const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                        two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                        Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                        Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
                        Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
    double hfsq, f, s, z, R, w, t1, t2, dk;
    int32_t k, hx, i, j;
    uint32_t lx;
    hx = (int32_t)hi_word(x);
    lx = lo_word(x);
    k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | lx) == 0) return -two54 / 0.0;
        if (hx < 0) return (x - x) / 0.0;
        k -= 54;
        x *= two54;
        hx = (int32_t)hi_word(x);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    i = (hx + 0x95f64) & 0x100000;
    x = set_hi_word(x, (uint32_t)(hx | (i ^ 0x3ff00000)));
    k += (i >> 20);
    f = x - 1.0;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) {
            if (k == 0) return 0.0;
            dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    s = f / (2.0 + f);
    dk = (double)k;
    z = s * s;
    i = hx - 0x6147a;
    w = z * z;
    j = 0x6b851 - hx;
    t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    R = t2 + t1;
    if (i > 0) {
        hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

double fpc_log10(double x) { return fpc_ln(x) * 0.43429448190325182765; }

long long fpc_round(double x) { return (long long)nearbyint(x); }

long long fpc_ceil(double x) {
    double t = trunc(x);
    long long r = (long long)t;
    if (x - t > 0.0) r += 1;
    return r;
}

int fpc_iszero(double x) { return fabs(x) <= 1e-12; }
