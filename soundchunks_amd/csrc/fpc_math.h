// FPC 3.2.2 (Win64) RTL numerics the encoder's features depend on, restated
// for the product host runtime.  Feature arguments form finite sets
// (CS^2 DCT angles, CS^2 DFT angles) so the runtime evaluates these once per
// chunk size into tables; the per-chunk work is table-driven.
//   sin/cos: Cephes kernels + FPC rem_pio2 (encoder.exe @0x10000b9f0,
//            @0x10000bb40, reduction @0x10000b150, fdlibm k_rem_pio2 @0x10000a500)
//   ln:      fdlibm e_log (encoder.exe @0x10000b690); log10 = ln * 1/ln(10)
#pragma once
#include <cstdint>

namespace gsc {
namespace fpc {

#if defined(__HIPCC__)
#define FPC_HD __host__ __device__
#else
#define FPC_HD
#endif

double sin(double x);
double cos(double x);

// fdlibm e_log as FPC 3.2.2 ships it (encoder.exe @0x10000b690); host and
// device evaluate the same IEEE f64 operation sequence (-ffp-contract=off)
FPC_HD inline double ln(double x) {
    constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                     two54 = 1.80143985094819840000e+16;
    constexpr double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                     Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                     Lg7 = 1.479819860511658591e-01;
    uint64_t u = __builtin_bit_cast(uint64_t, x);
    int32_t hx = int32_t(uint32_t(u >> 32));
    const uint32_t lx = uint32_t(u);
    int32_t k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | int32_t(lx)) == 0) return -two54 / 0.0;
        if (hx < 0) return (x - x) / 0.0;
        k -= 54;
        x *= two54;
        hx = int32_t(uint32_t(__builtin_bit_cast(uint64_t, x) >> 32));
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    int32_t i = (hx + 0x95f64) & 0x100000;
    u = __builtin_bit_cast(uint64_t, x);
    u = (u & 0xffffffffull) | (uint64_t(uint32_t(hx | (i ^ 0x3ff00000))) << 32);
    x = __builtin_bit_cast(double, u);
    k += i >> 20;
    const double f = x - 1.0;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) {
            if (k == 0) return 0.0;
            const double dk = double(k);
            return dk * ln2_hi + dk * ln2_lo;
        }
        const double R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        const double dk = double(k);
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    const double s = f / (2.0 + f);
    const double dk = double(k);
    const double z = s * s;
    i = hx - 0x6147a;
    const double w = z * z;
    const int32_t j = 0x6b851 - hx;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    const double R = t2 + t1;
    if (i > 0) {
        const double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}
FPC_HD inline double log10(double x) { return ln(x) * 0.43429448190325182765; }
// FPC round(): cvtsd2si, round half to even
int64_t round(double x);
// FPC math.ceil for the non-negative arguments used here
int64_t ceil_pos(double x);
FPC_HD inline bool is_zero(double x) { return (x < 0 ? -x : x) <= 1e-12; }

}  // namespace fpc
}  // namespace gsc
