// Exact-integer applies of a phase-code sensing matrix on the int8 matrix cores
// (v_mfma_i32_32x32x32_i8), for the r = 1 ADMM iteration with one shared codebook:
//
//   apply_A   T = S - A V        S = Y - M/mu,  V = Z - N/mu   (ArgMinX residual, :325-330)
//   apply_AH  X = V + A^H g                                    (ArgMinX, :325)
//
// The codebooks of the reference are phase codes: random_probe_cb_*.mat and
// Random_Phase_State hold entries in {+-1, +-j} (times one common factor after the
// normalisation of inferLowRankV4_multi.m:27-38), the multiresolution codebooks add
// switched-off antennas (0).  Every real component of such an A is in {0, +-c}.  Then
//
//   A v = c (P + jQ)(v_r + j v_i),  P, Q in {-1, 0, 1}^(m x n)
//
// is an integer combination of the entries of v.  Each realisation's vector is cut into
// fixed-point digits against one power-of-two exponent 2^e >= max|component| (the
// Ozaki scheme): w = rint(v 2^(54-e)) is a 56-bit integer, written as seven unsigned
// 7-bit digits and a signed top digit, w = sum_t u_t 128^t.  The 2x2 real expansion of
// P + jQ times every digit plane is an exact int8 x int8 -> int32 product (|partial| <=
// 127 * 2n < 2^31), and the planes are recombined in f64 (Horner, most significant
// first).  The only rounding beyond the f64 epilogue is the truncation of v to 2^(e-55),
// i.e. the result carries an f64 GEMM's accuracy (relative error ~1e-16 of max|v|).
//
// GEMM shape: rows = (realisation, digit) pairs, 16 realisations x 8 digits = 128 rows
// per work-group; cols = output reals (512 per work-group, 8 waves x 2 tiles of 32);
// K = 2 x (complex inner dimension), staged 128 reals at a time.  The digit planes are
// formed while staging (f64 -> int digits in VGPRs -> LDS); the int8 codebook is read
// in fragment order straight from global memory (1 KiB per wave per tile and K-step,
// coalesced) two K-steps ahead.  A 32-row MFMA tile holds 4 realisations x 8 digits,
// arranged so that each lane's accumulator registers 0..7 / 8..15 are the 8 digit planes
// of one realisation at one output column: the recombination needs no data movement.
//
// Exponents: apply_A takes max|V| from the Z-step (RealState::vbound, a rigorous upper
// bound |Z| + |N|/mu formed as Z and N are written); apply_AH takes max|g| over the
// realisation's m entries in a pre-pass.  A non-finite bound yields NaN outputs for that
// realisation (the f64 product would not be finite either).
#include "ace_common.hpp"

#include <cfloat>

namespace ace {

namespace {
typedef int i4v __attribute__((ext_vector_type(4)));
typedef int i16v __attribute__((ext_vector_type(16)));

constexpr int RB = 16;           // realisations per work-group
constexpr int ROWS = RB * 8;     // MFMA rows per work-group (realisation, digit)
constexpr int KC = 128;          // K reals per stage
constexpr int RS = KC + 16;      // LDS row stride (bytes): 16-byte slots of 8 consecutive rows distinct
constexpr int NCB = 512;         // output reals per work-group
constexpr int NT = 512;          // threads (8 waves)
constexpr int KSC = KC / 32;     // MFMA K-steps per stage

// LDS row of (realisation bl in 0..15, digit t in 0..7): inverse of the accumulator map
// row = (g & 3) + 8 (g >> 2) + 4 h  ->  realisation 4R + 2 (g >> 3) + h, digit (g & 3) + 4 ((g >> 2) & 1)
__device__ __forceinline__ int lds_row(int bl, int t) {
    const int R = bl >> 2, q = (bl >> 1) & 1, h = bl & 1;
    return 32 * R + 16 * q + 8 * (t >> 2) + 4 * h + (t & 3);
}

// Fixed-point digits of 2 complex entries (4 reals) as 8 packed dwords (byte i = real i).
__device__ __forceinline__ void digits4(const double (&v)[4], double p2, uint32_t (&out)[8]) {
    uint32_t lo[4];
    int32_t hi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double x = rint(v[i] * p2);             // |x| < 2^55 (2^54 nominal)
        const double h = floor(x * 0x1p-32);
        const double l = fma(-h, 0x1p32, x);          // [0, 2^32), exact
        hi[i] = (int32_t)h;
        lo[i] = (uint32_t)l;
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        uint32_t d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (t < 4) d[i] = (lo[i] >> (7 * t)) & 127u;
            else if (t == 4) d[i] = __builtin_amdgcn_alignbit((uint32_t)hi[i], lo[i], 28) & 127u;
            else if (t == 5) d[i] = ((uint32_t)hi[i] >> 3) & 127u;
            else if (t == 6) d[i] = ((uint32_t)hi[i] >> 10) & 127u;
            else d[i] = (uint32_t)(hi[i] >> 17) & 255u;   // signed top digit
        }
        out[t] = d[0] | (d[1] << 8) | (d[2] << 16) | (d[3] << 24);
    }
}

__device__ __forceinline__ int exp_of(double bound) {
    int e = bound > 0.0 ? ilogb(bound) + 1 : 0;
    return e < -960 ? -960 : (e > 1000 ? 1000 : e);
}

// MODE 1: C = E1 - E2/mu - c (A V),  V = V1 - V2/mu   (K = n, outputs m)
// MODE 2: C = E1 - E2/mu + c (A^H V), V = V1           (K = m, outputs n)
template <int MODE>
__global__ __launch_bounds__(NT, 1) void i8apply_kernel(int nb, int Kc, int Mc, int nks, const i4v* __restrict__ Bf,
                                                        const double* __restrict__ V1, const double* __restrict__ V2,
                                                        const double* __restrict__ E1, const double* __restrict__ E2,
                                                        double* __restrict__ C, const double* __restrict__ cptr,
                                                        const RealState* __restrict__ rs) {
    __shared__ __attribute__((aligned(16))) int8_t As[2][ROWS * RS];
    __shared__ double sc_s[RB], imu_s[RB];
    __shared__ int live_s[RB];

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int j0 = blockIdx.x * RB, cb = blockIdx.y;
    // staging role: realisation bl, complex pair cp (entries 64 kc + 2 cp, +1 of chunk kc)
    const int bl = t >> 5, cp = t & 31, jb = j0 + bl;
    const bool live = jb < nb && !rs[jb].done;
    const double imu = live ? 1.0 / rs[jb].mu : 0.0;
    const d2* v1 = reinterpret_cast<const d2*>(V1) + (long long)jb * Kc;
    const d2* v2 = reinterpret_cast<const d2*>(V2) + (long long)jb * Kc;

    double bound = 0.0;
    if (MODE == 1) {
        bound = live ? rs[jb].vbound : 0.0;
    } else {   // max |g| over the realisation (32 lanes of this half-wave)
        double mx = 0.0, sn = 0.0;
        if (live)
            for (int k = cp; k < Kc; k += 32) {
                const d2 v = v1[k];
                const double ax = fabs(v.x), ay = fabs(v.y);
                mx = fmax(mx, fmax(ax, ay));
                sn += 0.0 * (ax + ay);   // NaN / Inf sticky
            }
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
            mx = fmax(mx, __shfl_xor(mx, o, 64));
            sn += __shfl_xor(sn, o, 64);
        }
        bound = mx + sn;
    }
    const bool finite = bound <= DBL_MAX;
    const int e = finite ? exp_of(bound) : 0;
    const double p2 = ldexp(1.0, 54 - e);
    if (cp == 0) {
        sc_s[bl] = finite ? (*cptr) * ldexp(1.0, e - 54) : __builtin_nan("");
        imu_s[bl] = imu;
        live_s[bl] = live;
    }

    // ---- staging: 2 complex entries of realisation bl per thread per stage
    d2 g1[2], g2[2];
    auto gload = [&](int kc) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k = KC / 2 * kc + 2 * cp + u;
            g1[u] = g2[u] = make_double2(0.0, 0.0);
            if (live && k < Kc) {
                g1[u] = v1[k];
                if (MODE == 1) g2[u] = v2[k];
            }
        }
    };
    auto lstore = [&](int buf) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            d2 x = g1[u];
            if (MODE == 1) x = make_double2(fma(-g2[u].x, imu, x.x), fma(-g2[u].y, imu, x.y));   // V = Z - N/mu (xw)
            v[2 * u] = x.x;
            v[2 * u + 1] = x.y;
        }
        uint32_t d[8];
        digits4(v, p2, d);
#pragma unroll
        for (int tt = 0; tt < 8; ++tt)
            *reinterpret_cast<uint32_t*>(&As[buf][lds_row(bl, tt) * RS + 4 * cp]) = d[tt];
    };

    // ---- codebook fragments: wave w owns column tiles ct0, ct0 + 1 of the 32-column tiles
    const int ct0 = cb * (NCB / 32) + 2 * w;
    const i4v* bp0 = Bf + (long long)ct0 * nks * 64 + lane;
    const i4v* bp1 = bp0 + (long long)nks * 64;
    // three-deep register ring (current, +1, +2 K-steps), rotated by value
    i4v bc0, bc1, bn0, bn1, bm0, bm1;

    i16v acc[4][2];
#pragma unroll
    for (int R = 0; R < 4; ++R)
#pragma unroll
        for (int c = 0; c < 2; ++c) acc[R][c] = i16v{};

    const int nstage = nks / KSC;
    bc0 = bp0[0];
    bc1 = bp1[0];
    bn0 = bp0[64];
    bn1 = bp1[64];
    gload(0);
    lstore(0);
    __syncthreads();
    const int8_t* arow = nullptr;
    for (int s = 0; s < nstage; ++s) {
        const int buf = s & 1;
        if (s + 1 < nstage) gload(s + 1);
        arow = &As[buf][(lane & 31) * RS + 16 * (lane >> 5)];
#pragma unroll
        for (int kk = 0; kk < KSC; ++kk) {
            const int ks = s * KSC + kk;
            if (ks + 2 < nks) {
                bm0 = bp0[(long long)(ks + 2) * 64];
                bm1 = bp1[(long long)(ks + 2) * 64];
            }
            i4v af[4];
#pragma unroll
            for (int R = 0; R < 4; ++R) af[R] = *reinterpret_cast<const i4v*>(arow + 32 * R * RS + 32 * kk);
#pragma unroll
            for (int R = 0; R < 4; ++R) {
                acc[R][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[R], bc0, acc[R][0], 0, 0, 0);
                acc[R][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[R], bc1, acc[R][1], 0, 0, 0);
            }
            bc0 = bn0;
            bc1 = bn1;
            bn0 = bm0;
            bn1 = bm1;
        }
        if (s + 1 < nstage) lstore(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue: lane (col = lane & 31, h = lane >> 5), registers 8q..8q+7 = digits of
    // realisation 4R + 2q + h
    const int h = lane >> 5;
    const int ldo = 2 * Mc;   // reals per output row
#pragma unroll
    for (int R = 0; R < 4; ++R)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int blo = 4 * R + 2 * q + h, j = j0 + blo;
            if (j >= nb || !live_s[blo]) continue;
            const double sc = sc_s[blo], im = imu_s[blo];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int col = (ct0 + c) * 32 + (lane & 31);
                if (col >= ldo) continue;
                double a = (double)acc[R][c][8 * q + 7];
#pragma unroll
                for (int tt = 6; tt >= 0; --tt) a = fma(a, 128.0, (double)acc[R][c][8 * q + tt]);
                const long long off = (long long)j * ldo + col;
                if (MODE == 2 && !E1) {   // raw product W for the Z-step's wmode
                    C[off] = sc * a;
                    continue;
                }
                const double ev = fma(-E2[off], im, E1[off]);
                C[off] = MODE == 1 ? ev - sc * a : ev + sc * a;
            }
        }
}

// Codebook check and expansion.  cmax = max |component| of A (device scalar).  Each
// complex entry A[i][k] = c (p + j q) must have p, q in {-1, 0, 1}; flag is set otherwise.
//   apply_A  (cols 2m, K 2n):  L[2i][2k] = p, L[2i][2k+1] = -q, L[2i+1][2k] = q, L[2i+1][2k+1] = p
//   apply_AH (cols 2n, K 2m):  H[2k][2i] = p, H[2k][2i+1] = q, H[2k+1][2i] = -q, H[2k+1][2i+1] = p
// Fragment order: byte (col, k) of a [cols][K] matrix at ((col/32 * nks + k/32) * 64 + col%32 +
// 32 ((k%32)/16)) * 16 + k%16  (lane l of an MFMA operand holds col l&31, k 16 (l>>5) .. +15).
__device__ __forceinline__ long long frag_off(int col, int k, int nks) {
    return ((long long)((col >> 5) * nks + (k >> 5)) * 64 + (col & 31) + 32 * ((k & 31) >> 4)) * 16 + (k & 15);
}
__global__ __launch_bounds__(256) void i8_expand_kernel(int m, int n, const double* __restrict__ Ap,
                                                         const double* __restrict__ cmax, int8_t* __restrict__ LA,
                                                         int nksA, int8_t* __restrict__ LH, int nksH, int* flag) {
    const long long e = blockIdx.x * 256LL + threadIdx.x;
    if (e >= (long long)m * n) return;
    const int i = (int)(e / n), k = (int)(e % n);
    const d2 a = reinterpret_cast<const d2*>(Ap)[e];
    const double c = *cmax;
    auto code = [&](double x, int& ok) -> int {
        if (x == c) return 1;
        if (x == -c) return -1;
        if (x == 0.0) return 0;
        ok = 0;
        return 0;
    };
    int ok = 1;
    const int p = code(a.x, ok), q = code(a.y, ok);
    if (!ok) atomicOr(flag, 1);
    LA[frag_off(2 * i, 2 * k, nksA)] = (int8_t)p;
    LA[frag_off(2 * i, 2 * k + 1, nksA)] = (int8_t)(-q);
    LA[frag_off(2 * i + 1, 2 * k, nksA)] = (int8_t)q;
    LA[frag_off(2 * i + 1, 2 * k + 1, nksA)] = (int8_t)p;
    LH[frag_off(2 * k, 2 * i, nksH)] = (int8_t)p;
    LH[frag_off(2 * k, 2 * i + 1, nksH)] = (int8_t)q;
    LH[frag_off(2 * k + 1, 2 * i, nksH)] = (int8_t)(-q);
    LH[frag_off(2 * k + 1, 2 * i + 1, nksH)] = (int8_t)p;
}
}  // namespace

// padded K-steps (of 32 reals) for a complex inner dimension kc: multiple of one stage
int i8_nks(int kc) { return (2 * kc + KC - 1) / KC * KSC; }
// padded 32-column tiles for mc complex outputs: multiple of one work-group's 512 columns
int i8_ncols(int mc) { return (2 * mc + NCB - 1) / NCB * NCB; }
size_t i8_frag_bytes(int mc, int kc) { return (size_t)i8_ncols(mc) * i8_nks(kc) * 32; }

void launch_i8_expand(int m, int n, const double* A, const double* cmax, int8_t* LA, int8_t* LH, int* flag,
                      hipStream_t st) {
    const long long tot = (long long)m * n;
    hipLaunchKernelGGL(i8_expand_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, m, n, A, cmax, LA,
                       i8_nks(n), LH, i8_nks(m), flag);
}

void launch_i8_apply(int mode, int nb, int Kc, int Mc, const int8_t* Bfrag, const double* V1, const double* V2,
                     const double* E1, const double* E2, double* C, const double* cmax, const RealState* rs,
                     hipStream_t st) {
    dim3 grid((nb + RB - 1) / RB, i8_ncols(Mc) / NCB, 1), block(NT);
    const i4v* B = reinterpret_cast<const i4v*>(Bfrag);
    if (mode == 1)
        hipLaunchKernelGGL(i8apply_kernel<1>, grid, block, 0, st, nb, Kc, Mc, i8_nks(Kc), B, V1, V2, E1, E2, C, cmax,
                           rs);
    else
        hipLaunchKernelGGL(i8apply_kernel<2>, grid, block, 0, st, nb, Kc, Mc, i8_nks(Kc), B, V1, V2, E1, E2, C, cmax,
                           rs);
}

}  // namespace ace
