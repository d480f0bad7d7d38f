// Shared pieces of the exact int8 digit-plane applies (ace_i8gemm.hip: one shared codebook;
// ace_private.hip: one codebook per realisation): the fixed-point digit scheme and the
// v_mfma_i32_32x32x32_i8 accumulator map.
//
// Digits (Ozaki scheme): a vector is cut against one power-of-two exponent 2^e >= max|component|:
// w = rint(v 2^(54-e)) is a 56-bit integer written as seven unsigned 7-bit digits and a signed top
// digit, w = sum_t u_t 128^t.  A digit plane times an int8 {0, +-1} operand is an exact int32 product
// and the planes are recombined in f64 (Horner from the top digit), so the result carries an f64
// GEMM's accuracy.
#pragma once
#include "ace_common.hpp"

#include <cfloat>

namespace ace {
namespace {

typedef int i4v __attribute__((ext_vector_type(4)));
typedef int i16v __attribute__((ext_vector_type(16)));

// MFMA row of (slot bl in 0..15, digit t in 0..7) such that accumulator registers 8q..8q+7 of lane l
// are the 8 digit planes of slot 4R + 2q + (l >> 5) at output column l & 31: the inverse of the
// accumulator map row = (g & 3) + 8 (g >> 2) + 4 h  ->  slot 4R + 2 (g >> 3) + h, digit (g & 3) + 4 ((g >> 2) & 1)
__device__ __forceinline__ int lds_row(int bl, int t) {
    const int R = bl >> 2, q = (bl >> 1) & 1, h = bl & 1;
    return 32 * R + 16 * q + 8 * (t >> 2) + 4 * h + (t & 3);
}

__device__ __forceinline__ int exp_of(double bound) {
    int e = bound > 0.0 ? ilogb(bound) + 1 : 0;
    return e < -960 ? -960 : (e > 1000 ? 1000 : e);
}

// Recombined digit planes of output column col for slot 4R + 2q + (lane >> 5):
// sum_t acc[8q + t] 128^t (Horner from the signed top digit).
__device__ __forceinline__ double recombine(const i16v& a, int q) {
    double v = (double)a[8 * q + 7];
#pragma unroll
    for (int tt = 6; tt >= 0; --tt) v = fma(v, 128.0, (double)a[8 * q + tt]);
    return v;
}

// Exponent and scale of one vector's digit planes from a bound on max|component|.
__device__ __forceinline__ void plane_scale(double bound, double c, double& p2, double& sc) {
    const bool finite = bound <= DBL_MAX;
    const int e = finite ? exp_of(bound) : 0;
    p2 = ldexp(1.0, 54 - e);
    sc = finite ? c * ldexp(1.0, e - 54) : __builtin_nan("");
}

// The 8 digits (t = 0..7) of one real component x already scaled by p2 (|x| < 2^55): bytes of
// the 56-bit integer rint(x) as seven unsigned 7-bit digits and a signed top digit.
__device__ __forceinline__ void digits1(double xs, uint32_t (&d)[8]) {
    const double x = rint(xs);
    const double h = floor(x * 0x1p-32);
    const uint32_t lo = (uint32_t)fma(-h, 0x1p32, x);   // [0, 2^32), exact
    const int32_t hi = (int32_t)h;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        if (t < 4) d[t] = (lo >> (7 * t)) & 127u;
        else if (t == 4) d[t] = __builtin_amdgcn_alignbit((uint32_t)hi, lo, 28) & 127u;
        else if (t == 5) d[t] = ((uint32_t)hi >> 3) & 127u;
        else if (t == 6) d[t] = ((uint32_t)hi >> 10) & 127u;
        else d[t] = (uint32_t)(hi >> 17) & 255u;   // signed top digit
    }
}

}  // namespace
}  // namespace ace
