// Complex fp64 GEMM on the gfx950 f64 matrix cores (v_mfma_f64_16x16x4_f64) for the
// shared-codebook regime: one complex LHS (A, A^H, G or K; shared by the whole
// batch) times a panel of per-realisation vectors.
//
// Complex arithmetic is run as a real GEMM on the 2x2 real expansion of each
// complex LHS entry; the expansion happens on the fly while reading fragments
// from LDS, so the LHS is streamed as plain complex128.  State vectors are
// complex128 interleaved, realisation-major, so the real "K" index of the
// expansion (k' = 2k + {re,im}) is just the double index inside a vector.
//
//   D^T[j][i'] = sum_k' Vhat[j][k'] * Lhat[i'][k']     (j: realisation, i' = 2i + c)
//   Lhat[2i+c][2k+d] = c==d ? Re L_ik : (c==0 ? -Im L_ik : Im L_ik)
//
// MFMA operand maps (verified on MI355X with asymmetric data, tools/probe_fp64.hip):
//   A-frag lane l: A[row = l&15][k = l>>4];  B-frag: B[k = l>>4][col = l&15];
//   D lane l, reg r: D[row = (l>>4) + 4r][col = l&15].
// Here A = Vhat (rows = realisations), B = Lhat^T (cols = output reals), so each
// output row (one realisation) is written as 16 consecutive doubles = 128 B.
//
// Work-group tile: 64 realisations x 64 output reals (32 complex rows), K-step 32
// reals (16 complex); 4 waves in a 2x2 arrangement, each 2x2 MFMA tiles (4 f64
// accumulators).  LDS: V 2x64x34 doubles + L 2x32x17 complex = 52 KiB (3 WGs/CU).
// The block -> tile map is XCD-aware: blocks that share one V panel are dealt
// to the same XCD (blocks b and b+8 share an XCD under round-robin dispatch) so
// the panel is served from that XCD's L2.
#include "ace_common.hpp"

namespace ace {

namespace {
constexpr int BJ = 64;      // realisations per tile
constexpr int BI = 64;      // output reals per tile (32 complex rows)
constexpr int BK = 32;      // reals of K per step (16 complex)
constexpr int VST = BK + 2; // V row stride (doubles): 34 = 2 mod 32 -> conflict-free ds_read_b64 A-fragments
constexpr int LST = BK / 2 + 1; // L row stride (complex)

template <int MODE, bool CONJ_L>
__global__ __launch_bounds__(256) void zgemm_kernel(int M, int K, int nb, const double* __restrict__ L, int ldl,
                                                    long long strideL, const double* __restrict__ V, int ldv,
                                                    long long strideV, double* __restrict__ C,
                                                    const double* __restrict__ E, int ldc, long long strideC,
                                                    int tilesI, int tilesJ) {
    __shared__ double Vs[2][BJ * VST];
    __shared__ d2 Ls[2][(BI / 2) * LST];

    const int z = blockIdx.z;
    L += 2 * strideL * z;
    V += 2 * strideV * z;
    C += 2 * strideC * z;
    if (MODE != 0) E += 2 * strideC * z;

    // XCD-aware bijective remap of the linear block id.
    const int nblk = tilesI * tilesJ;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, local = bid >> 3;
    const int q = nblk >> 3, rr = nblk & 7;
    const int nid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + local;
    const int ti = nid % tilesI, tj = nid / tilesI;
    const int i0c = ti * (BI / 2);  // first complex output row
    const int j0 = tj * BJ;         // first realisation

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wj = w >> 1, wi = w & 1;

    // global -> register staging indices
    const int vj = t >> 2, vseg = (t & 3) * 8;      // V: realisation vj, reals vseg..vseg+7 of the K-step
    const int lr = t >> 3, lkc = (t & 7) * 2;       // L: complex row lr, complex cols lkc, lkc+1
    const int Kr = 2 * K;                           // reals of K
    const int ksteps = (Kr + BK - 1) / BK;
    const bool vrow_ok = (j0 + vj) < nb;
    const bool lrow_ok = (i0c + lr) < M;
    const double* vptr = V + 2LL * (long long)(j0 + vj) * ldv + vseg;
    const double* lptr = L + 2LL * ((long long)(i0c + lr) * ldl + lkc);

    double vreg[8];
    d2 lreg[2];
    // interior tiles (block-uniform) load without bounds checks
    const bool full = (j0 + BJ <= nb) && (i0c + BI / 2 <= M) && (Kr % BK == 0);
    auto gload = [&](int ks) {
        const int kb = ks * BK;
        if (full) {
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
                const d2 v = *reinterpret_cast<const d2*>(vptr + kb + e);
                vreg[e] = v.x;
                vreg[e + 1] = v.y;
            }
#pragma unroll
            for (int e = 0; e < 2; ++e) lreg[e] = *reinterpret_cast<const d2*>(lptr + 2LL * ((kb >> 1) + e));
            return;
        }
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
            const int kr = kb + vseg + e;
            d2 v = make_double2(0.0, 0.0);
            if (vrow_ok && kr < Kr) v = *reinterpret_cast<const d2*>(vptr + kb + e);
            vreg[e] = v.x;
            vreg[e + 1] = v.y;
        }
        const int kc = (kb >> 1) + lkc;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            d2 v = make_double2(0.0, 0.0);
            if (lrow_ok && kc + e < K) v = *reinterpret_cast<const d2*>(lptr + 2LL * ((kb >> 1) + e));
            lreg[e] = v;
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int e = 0; e < 8; ++e) Vs[buf][vj * VST + vseg + e] = vreg[e];
        Ls[buf][lr * LST + lkc] = lreg[0];
        Ls[buf][lr * LST + lkc + 1] = lreg[1];
    };

    d4v acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = d4v{0.0, 0.0, 0.0, 0.0};

    // per-lane constants of the on-the-fly complex -> 2x2 real expansion
    const int c_par = lane & 1;          // output real parity (re/im row)
    const int d_par = (lane >> 4) & 1;   // K real parity (re/im of the vector entry)
    const int sel = (c_par == d_par) ? 0 : 1;
    // sign of the expanded entry, applied as a sign-bit XOR (one VALU op)
    const bool neg = !CONJ_L ? (c_par == 0 && d_par == 1) : (c_par == 1 && d_par == 0);
    const long long smask = neg ? (long long)0x8000000000000000ULL : 0LL;

    gload(0);
    lstore(0);
    __syncthreads();

    for (int ks = 0; ks < ksteps; ++ks) {
        const int buf = ks & 1;
        if (ks + 1 < ksteps) gload(ks + 1);
        const double* vs = Vs[buf];
        const double* ls = reinterpret_cast<const double*>(Ls[buf]);
#pragma unroll
        for (int kk = 0; kk < BK / 4; ++kk) {
            const int kr = kk * 4 + (lane >> 4);
            double af[2], bf[2];
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) af[jj] = vs[(wj * 32 + jj * 16 + (lane & 15)) * VST + kr];
#pragma unroll
            for (int ii = 0; ii < 2; ++ii) {
                const int ir = wi * 32 + ii * 16 + (lane & 15);
                bf[ii] = __longlong_as_double(__double_as_longlong(ls[2 * ((ir >> 1) * LST + (kr >> 1)) + sel]) ^ smask);
            }
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                for (int ii = 0; ii < 2; ++ii)
                    acc[jj][ii] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[jj], bf[ii], acc[jj][ii], 0, 0, 0);
        }
        if (ks + 1 < ksteps) lstore(buf ^ 1);
        __syncthreads();
    }

    // epilogue: lane l, reg r -> realisation j0 + wj*32 + jj*16 + (l>>4) + 4r, real i0' + wi*32 + ii*16 + (l&15)
    const int Mr = 2 * M;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = j0 + wj * 32 + jj * 16 + (lane >> 4) + 4 * r;
                const int ir = 2 * i0c + wi * 32 + ii * 16 + (lane & 15);
                if (j < nb && ir < Mr) {
                    const long long off = 2LL * (long long)j * ldc + ir;
                    double v = acc[jj][ii][r];
                    if (MODE == 1) v = E[off] - v;
                    else if (MODE == 2) v = E[off] + v;
                    C[off] = v;
                }
            }
}
}  // namespace

void launch_zgemm(int mode, bool conj_l, int M, int K, int nb, const double* L, int ldl, long long strideL,
                  const double* V, int ldv, long long strideV, double* C, const double* E, int ldc,
                  long long strideC, int nz, hipStream_t st) {
    const int tilesI = (M + BI / 2 - 1) / (BI / 2);
    const int tilesJ = (nb + BJ - 1) / BJ;
    dim3 grid(tilesI * tilesJ, 1, nz), block(256);
#define ACE_GEMM_LAUNCH(MD, CJ)                                                                              \
    hipLaunchKernelGGL((zgemm_kernel<MD, CJ>), grid, block, 0, st, M, K, nb, L, ldl, strideL, V, ldv, strideV, \
                       C, E, ldc, strideC, tilesI, tilesJ)
    if (conj_l) {
        if (mode == 0) ACE_GEMM_LAUNCH(0, true);
        else if (mode == 1) ACE_GEMM_LAUNCH(1, true);
        else ACE_GEMM_LAUNCH(2, true);
    } else {
        if (mode == 0) ACE_GEMM_LAUNCH(0, false);
        else if (mode == 1) ACE_GEMM_LAUNCH(1, false);
        else ACE_GEMM_LAUNCH(2, false);
    }
#undef ACE_GEMM_LAUNCH
}

}  // namespace ace
