/*
 * ORACLE (test infrastructure only) -- CPU restatement of the Free Pascal 3.2.2
 * Win64 RTL numerics that the reference encoder's hot path depends on.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
 * anything under oracle/.  The product library never links this file.
 *
 * Pinning: the restatement follows the disassembly of reference
 * encoder/encoder.exe (read as text, never executed):
 *   sin      @0x10000b9f0, cos @0x10000bb40, reduction @0x10000b150,
 *   polevl   @0x10000a480, floor @0x10000a4b0, kernel_rem_pio2 @0x10000a500,
 *   ln       @0x10000b690 (fdlibm e_log), log10 = ln * 0.4342944819032518
 *            (@0x10003eeda).
 * The two_over_pi table and every polynomial constant are checked against
 * mpmath / the fdlibm literals in tests/test_oracle_fpc.py.
 */
#ifndef GSC_ORACLE_FPC_RTL_H
#define GSC_ORACLE_FPC_RTL_H

#ifdef __cplusplus
extern "C" {
#endif

double fpc_sin(double x);
double fpc_cos(double x);
double fpc_ln(double x);
double fpc_log10(double x);
/* rem_pio2 as FPC implements it: returns the quadrant (mod 8), *y = remainder */
long   fpc_rem_pio2(double x, double *y);
/* FPC round(): cvtsd2si under default MXCSR = round half to even */
long long fpc_round(double x);
/* FPC math.ceil (returns integer): trunc, +1 if frac > 0 */
long long fpc_ceil(double x);
/* FPC IsZero(Double): |x| <= 1e-12 */
int fpc_iszero(double x);

#ifdef __cplusplus
}
#endif
#endif
