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

double sin(double x);
double cos(double x);
double ln(double x);
inline double log10(double x) { return ln(x) * 0.43429448190325182765; }
// FPC round(): cvtsd2si, round half to even
int64_t round(double x);
// FPC math.ceil for the non-negative arguments used here
int64_t ceil_pos(double x);
inline bool is_zero(double x) { return (x < 0 ? -x : x) <= 1e-12; }

}  // namespace fpc
}  // namespace gsc
