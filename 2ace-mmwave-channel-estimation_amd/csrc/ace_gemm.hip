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

// Tile configuration: BJ realisations x BI output reals per work-group, BK reals of K per
// step, WJ x WI waves, each wave (BJ/WJ) x (BI/WI) reals = TJ x TI MFMA tiles.
template <int BJ_, int BI_, int BK_, int WJ_, int WI_>
struct GemmCfg {
    static constexpr int BJ = BJ_, BI = BI_, BK = BK_, WJ = WJ_, WI = WI_;
    static constexpr int NT = 64 * WJ * WI;
    static constexpr int TJ = BJ / WJ / 16, TI = BI / WI / 16;
    static constexpr int VST = BK + 2;      // V row stride (doubles): = 2 mod 32 -> conflict-free A-fragments
    static constexpr int LST = BK / 2 + 1;  // L row stride (complex)
    static constexpr int PV = BJ * (BK / 2) / NT;        // V complex pairs staged per thread per step
    static constexpr int PL = (BI / 2) * (BK / 2) / NT;  // L complex entries staged per thread per step
    static_assert(TJ >= 1 && TI >= 1 && BJ % (16 * WJ) == 0 && BI % (16 * WI) == 0, "wave tile");
    static_assert(PV >= 1 && PL >= 1 && BJ * (BK / 2) % NT == 0 && (BI / 2) * (BK / 2) % NT == 0, "staging");
    static_assert(BK % 4 == 0, "K step");
    static constexpr size_t lds_bytes() { return 2 * (size_t)BJ * VST * 8 + 2 * (size_t)(BI / 2) * LST * 16; }
};
using GemmDefault = GemmCfg<64, 64, 32, 2, 2>;

namespace {

template <int MODE, bool CONJ_L, class CF>
__global__ __launch_bounds__(CF::NT) void zgemm_kernel(int M, int K, int nb, const double* __restrict__ L, int ldl,
                                                       long long strideL, const double* __restrict__ V, int ldv,
                                                       long long strideV, double* __restrict__ C,
                                                       const double* __restrict__ E, int ldc, long long strideC,
                                                       int tilesI, int tilesJ) {
    constexpr int BJ = CF::BJ, BI = CF::BI, BK = CF::BK, NT = CF::NT, TJ = CF::TJ, TI = CF::TI;
    constexpr int VST = CF::VST, LST = CF::LST, PV = CF::PV, PL = CF::PL;
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
    const int wj = w / CF::WI, wi = w % CF::WI;
    const int Kr = 2 * K;  // reals of K
    const int ksteps = (Kr + BK - 1) / BK;

    double vreg[PV][2];
    d2 lreg[PL];
    // interior tiles (block-uniform) load without bounds checks
    const bool full = (j0 + BJ <= nb) && (i0c + BI / 2 <= M) && (Kr % BK == 0);
    auto gload = [&](int ks) {
        const int kb = ks * BK;
#pragma unroll
        for (int u = 0; u < PV; ++u) {
            const int p = t + NT * u, vj = p / (BK / 2), vs = 2 * (p % (BK / 2));
            d2 v = make_double2(0.0, 0.0);
            if (full || ((j0 + vj) < nb && kb + vs < Kr))
                v = *reinterpret_cast<const d2*>(V + 2LL * (long long)(j0 + vj) * ldv + kb + vs);
            vreg[u][0] = v.x;
            vreg[u][1] = v.y;
        }
#pragma unroll
        for (int u = 0; u < PL; ++u) {
            const int p = t + NT * u, lr = p / (BK / 2), lc = p % (BK / 2);
            const int kc = (kb >> 1) + lc;
            d2 v = make_double2(0.0, 0.0);
            if (full || ((i0c + lr) < M && kc < K))
                v = *reinterpret_cast<const d2*>(L + 2LL * ((long long)(i0c + lr) * ldl + kc));
            lreg[u] = v;
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int u = 0; u < PV; ++u) {
            const int p = t + NT * u, vj = p / (BK / 2), vs = 2 * (p % (BK / 2));
            Vs[buf][vj * VST + vs] = vreg[u][0];
            Vs[buf][vj * VST + vs + 1] = vreg[u][1];
        }
#pragma unroll
        for (int u = 0; u < PL; ++u) {
            const int p = t + NT * u, lr = p / (BK / 2), lc = p % (BK / 2);
            Ls[buf][lr * LST + lc] = lreg[u];
        }
    };

    d4v acc[TJ][TI];
#pragma unroll
    for (int a = 0; a < TJ; ++a)
#pragma unroll
        for (int b = 0; b < TI; ++b) acc[a][b] = d4v{0.0, 0.0, 0.0, 0.0};

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
            double af[TJ], bf[TI];
#pragma unroll
            for (int jj = 0; jj < TJ; ++jj) af[jj] = vs[(wj * (BJ / CF::WJ) + jj * 16 + (lane & 15)) * VST + kr];
#pragma unroll
            for (int ii = 0; ii < TI; ++ii) {
                const int ir = wi * (BI / CF::WI) + ii * 16 + (lane & 15);
                bf[ii] = __longlong_as_double(__double_as_longlong(ls[2 * ((ir >> 1) * LST + (kr >> 1)) + sel]) ^ smask);
            }
#pragma unroll
            for (int jj = 0; jj < TJ; ++jj)
#pragma unroll
                for (int ii = 0; ii < TI; ++ii)
                    acc[jj][ii] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[jj], bf[ii], acc[jj][ii], 0, 0, 0);
        }
        if (ks + 1 < ksteps) lstore(buf ^ 1);
        __syncthreads();
    }

    // epilogue: lane l, reg r -> realisation j0 + wj*(BJ/WJ) + jj*16 + (l>>4) + 4r, real i0' + wi*(BI/WI) + ii*16 + (l&15)
    const int Mr = 2 * M;
#pragma unroll
    for (int jj = 0; jj < TJ; ++jj)
#pragma unroll
        for (int ii = 0; ii < TI; ++ii)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = j0 + wj * (BJ / CF::WJ) + jj * 16 + (lane >> 4) + 4 * r;
                const int ir = 2 * i0c + wi * (BI / CF::WI) + ii * 16 + (lane & 15);
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

// ---- 3M variant (Gauss): (Vr + iVi)(Lr + iLi) from three real products
//   P1 = Vr Lr,  P2 = Vi Li,  P3 = (Vr + Vi)(Lr + Li);   Re = P1 - P2,  Im = P3 - P1 - P2
// (Li -> -Li for a conjugated L).  6 real flops per complex MAC instead of 8: three f64
// MFMAs per 16x16 complex block and 4 complex K instead of four.  The operands are read from
// LDS as whole complex numbers (one 16-byte read per fragment) and the two sums are formed in
// registers.  Tile: BJ realisations x BC complex outputs, BKC complex K per step, WJ x WI waves.
template <int BJ_, int BC_, int BKC_, int WJ_, int WI_>
struct Gemm3mCfg {
    static constexpr int BJ = BJ_, BC = BC_, BKC = BKC_, WJ = WJ_, WI = WI_;
    static constexpr int NT = 64 * WJ * WI;
    static constexpr int TJ = BJ / WJ / 16, TC = BC / WI / 16;
    static constexpr int VST = BKC + 1, LST = BKC + 1;  // complex row strides (odd)
    static constexpr int PV = BJ * BKC / NT, PL = BC * BKC / NT;
    static_assert(TJ >= 1 && TC >= 1 && BJ % (16 * WJ) == 0 && BC % (16 * WI) == 0, "wave tile");
    static_assert(PV >= 1 && PL >= 1 && BJ * BKC % NT == 0 && BC * BKC % NT == 0, "staging");
    static_assert(BKC % 4 == 0, "K step");
    static constexpr size_t lds_bytes() { return 2 * (size_t)(BJ * VST + BC * LST) * 16; }
};

namespace {

// FV: the V operand is formed while staging as V - V2 / mu_j (pre_kernel's V = Z - N/mu);
// FE: the epilogue operand is E - E2 / mu_j (S = Y - M/mu, or V = Z - N/mu), and rows of
// realisations already marked done are left untouched (as the unfused path leaves them).
// mu_j and done come from the per-realisation RealState array rs.
// YS (MODE 0, r = 1): the Y-step of ystep_kernel runs on the g tile in the epilogue; its five
// reductions are summed over the tile's outputs (16 lanes, then the WI waves, fixed order)
// and stored as the partial of (realisation, output tile).
template <int MODE, bool CONJ_L, class CF, bool FV = false, bool FE = false, bool YS = false>
__global__ __launch_bounds__(CF::NT) void zgemm3m_kernel(int M, int K, int nb, const double* __restrict__ L, int ldl,
                                                         long long strideL, const double* __restrict__ V, int ldv,
                                                         long long strideV, double* __restrict__ C,
                                                         const double* __restrict__ E, int ldc, long long strideC,
                                                         int tilesI, int tilesJ, const double* __restrict__ V2,
                                                         const double* __restrict__ E2, const RealState* __restrict__ rs,
                                                         YsArgs ys = YsArgs{}, const double* __restrict__ klim = nullptr,
                                                         long long klim_stride = 0) {
    constexpr int BJ = CF::BJ, BC = CF::BC, BKC = CF::BKC, NT = CF::NT, TJ = CF::TJ, TC = CF::TC;
    constexpr int VST = CF::VST, LST = CF::LST, PV = CF::PV, PL = CF::PL;
    __shared__ d2 Vs[2][BJ * VST];
    __shared__ d2 Ls[2][BC * LST];

    const int z = blockIdx.z;
    L += 2 * strideL * z;
    V += 2 * strideV * z;
    C += 2 * strideC * z;
    if (MODE != 0) E += 2 * strideC * z;

    const int nblk = tilesI * tilesJ;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, local = bid >> 3;
    const int q = nblk >> 3, rr = nblk & 7;
    const int nid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + local;
    const int ti = nid % tilesI, tj = nid / tilesI;
    const int i0 = ti * BC;  // first complex output
    const int j0 = tj * BJ;  // first realisation

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wj = w / CF::WI, wi = w % CF::WI;
    // klim (optional): per z-slice bound on the summation index (entries at or beyond it are zero in both operands,
    // e.g. PhaseLift's assembly over the kept eigenpairs): the K blocks past it are skipped
    if (klim) K = min(K, max(0, (int)klim[(long long)z * klim_stride]));
    const int ksteps = (K + BKC - 1) / BKC;

    d2 vreg[PV], lreg[PL];
    d2 v2reg[FV ? PV : 1];
    double vimu[FV ? PV : 1];
    if constexpr (FV) {
#pragma unroll
        for (int u = 0; u < PV; ++u) {
            const int j = j0 + (t + NT * u) / BKC;
            vimu[u] = j < nb ? 1.0 / rs[j].mu : 0.0;
        }
    }
    const bool full = (j0 + BJ <= nb) && (i0 + BC <= M) && (K % BKC == 0);
    auto gload = [&](int ks) {
        const int kb = ks * BKC;
#pragma unroll
        for (int u = 0; u < PV; ++u) {
            const int p = t + NT * u, vj = p / BKC, vc = p % BKC;
            d2 v = make_double2(0.0, 0.0), v2 = v;
            if (full || ((j0 + vj) < nb && kb + vc < K)) {
                v = *reinterpret_cast<const d2*>(V + 2LL * ((long long)(j0 + vj) * ldv + kb + vc));
                if constexpr (FV) v2 = *reinterpret_cast<const d2*>(V2 + 2LL * ((long long)(j0 + vj) * ldv + kb + vc));
            }
            vreg[u] = v;
            if constexpr (FV) v2reg[u] = v2;
        }
#pragma unroll
        for (int u = 0; u < PL; ++u) {
            const int p = t + NT * u, lr = p / BKC, lc = p % BKC;
            d2 v = make_double2(0.0, 0.0);
            if (full || ((i0 + lr) < M && kb + lc < K))
                v = *reinterpret_cast<const d2*>(L + 2LL * ((long long)(i0 + lr) * ldl + kb + lc));
            lreg[u] = v;
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int u = 0; u < PV; ++u) {
            const int p = t + NT * u;
            d2 v = vreg[u];
            if constexpr (FV) v = csub(v, cscale(v2reg[u], vimu[u]));
            Vs[buf][(p / BKC) * VST + p % BKC] = v;
        }
#pragma unroll
        for (int u = 0; u < PL; ++u) {
            const int p = t + NT * u;
            Ls[buf][(p / BKC) * LST + p % BKC] = lreg[u];
        }
    };

    d4v p1[TJ][TC], p2[TJ][TC], p3[TJ][TC];
#pragma unroll
    for (int a = 0; a < TJ; ++a)
#pragma unroll
        for (int b = 0; b < TC; ++b) p1[a][b] = p2[a][b] = p3[a][b] = d4v{0.0, 0.0, 0.0, 0.0};

    gload(0);
    lstore(0);
    __syncthreads();

    for (int ks = 0; ks < ksteps; ++ks) {
        const int buf = ks & 1;
        if (ks + 1 < ksteps) gload(ks + 1);
        const d2* vs = Vs[buf];
        const d2* ls = Ls[buf];
#pragma unroll
        for (int kk = 0; kk < BKC / 4; ++kk) {
            const int k = kk * 4 + (lane >> 4);
            double ar[TJ], ai[TJ], as[TJ], br[TC], bi[TC], bs[TC];
#pragma unroll
            for (int jj = 0; jj < TJ; ++jj) {
                const d2 v = vs[(wj * (BJ / CF::WJ) + jj * 16 + (lane & 15)) * VST + k];
                ar[jj] = v.x;
                ai[jj] = v.y;
                as[jj] = v.x + v.y;
            }
#pragma unroll
            for (int cc = 0; cc < TC; ++cc) {
                const d2 l = ls[(wi * (BC / CF::WI) + cc * 16 + (lane & 15)) * LST + k];
                br[cc] = l.x;
                bi[cc] = CONJ_L ? -l.y : l.y;
                bs[cc] = l.x + bi[cc];
            }
#pragma unroll
            for (int jj = 0; jj < TJ; ++jj)
#pragma unroll
                for (int cc = 0; cc < TC; ++cc) {
                    p1[jj][cc] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[jj], br[cc], p1[jj][cc], 0, 0, 0);
                    p2[jj][cc] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[jj], bi[cc], p2[jj][cc], 0, 0, 0);
                    p3[jj][cc] = __builtin_amdgcn_mfma_f64_16x16x4f64(as[jj], bs[cc], p3[jj][cc], 0, 0, 0);
                }
        }
        if (ks + 1 < ksteps) lstore(buf ^ 1);
        __syncthreads();
    }

    // epilogue: lane l, reg r -> realisation j0 + wj*(BJ/WJ) + jj*16 + (l>>4) + 4r, output i0 + wi*(BC/WI) + cc*16 + (l&15)
    if constexpr (YS) {
        static_assert(MODE == 0 && TC == 1, "fused Y-step: g = G T with one 16-output block per wave");
        double* red = reinterpret_cast<double*>(Vs[0]);  // [BJ rows][WI][5], free after the main loop
#pragma unroll
        for (int jj = 0; jj < TJ; ++jj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int jl = wj * (BJ / CF::WJ) + jj * 16 + (lane >> 4) + 4 * r;
                const int j = j0 + jl;
                const int i = i0 + wi * (BC / CF::WI) + (lane & 15);
                const double a = p1[jj][0][r], b = p2[jj][0][r];
                const d2 gv = make_double2(a - b, p3[jj][0][r] - a - b);
                double v[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
                if (j < nb && i < M) {
                    const long long off = (long long)j * ldc + i;
                    reinterpret_cast<d2*>(C)[off] = gv;
                    if (!rs[j].done) {  // ystep_kernel, element i
                        const double mu = rs[j].mu, imu = 1.0 / mu;
                        const d2 mi = reinterpret_cast<const d2*>(ys.M)[off];
                        const d2 yo = reinterpret_cast<const d2*>(ys.Yo)[off];
                        const double Bi = ys.B[off];
                        const d2 ax = csub(csub(yo, cscale(mi, imu)), gv);
                        d2 c = cadd(ax, cscale(mi, imu));
                        double d = sqrt(cabs2(c));
                        if (d == 0.0) {  // ArgMinY zero guard (:516-520 / :524-528)
                            c = make_double2(1.0, 0.0);
                            d = 1.0;
                        }
                        const double f = (Bi / d + mu) / (1.0 + mu);
                        const d2 y = cscale(c, f);
                        const d2 jv = csub(ax, y);
                        reinterpret_cast<d2*>(ys.M)[off] = cadd(mi, cscale(jv, mu));
                        reinterpret_cast<d2*>(ys.Yn)[off] = y;
                        const double aax = sqrt(cabs2(ax)) - Bi;
                        v[0] = aax * aax;
                        v[1] = cabs2(ax);
                        v[2] = cabs2(y);
                        v[3] = cabs2(jv);
                        v[4] = cabs2(csub(y, yo));
                    }
                }
#pragma unroll
                for (int k = 0; k < 5; ++k) v[k] = bsum16(v[k]);
                if ((lane & 15) == 0) {
#pragma unroll
                    for (int k = 0; k < 5; ++k) red[(jl * CF::WI + wi) * 5 + k] = v[k];
                }
            }
        __syncthreads();
        if (t < BJ) {
            const int j = j0 + t;
            if (j < nb && !rs[j].done) {
#pragma unroll
                for (int k = 0; k < 5; ++k) {
                    double s = 0.0;
#pragma unroll
                    for (int q = 0; q < CF::WI; ++q) s += red[(t * CF::WI + q) * 5 + k];
                    ys.part[((long long)j * tilesI + ti) * 5 + k] = s;
                }
            }
        }
        return;
    }
#pragma unroll
    for (int jj = 0; jj < TJ; ++jj)
#pragma unroll
        for (int cc = 0; cc < TC; ++cc)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = j0 + wj * (BJ / CF::WJ) + jj * 16 + (lane >> 4) + 4 * r;
                const int i = i0 + wi * (BC / CF::WI) + cc * 16 + (lane & 15);
                if (j < nb && i < M) {
                    if constexpr (FE) {
                        if (rs[j].done) continue;
                    }
                    const long long off = 2LL * ((long long)j * ldc + i);
                    const double a = p1[jj][cc][r], b = p2[jj][cc][r];
                    d2 v = make_double2(a - b, p3[jj][cc][r] - a - b);
                    if (MODE != 0) {
                        d2 e = *reinterpret_cast<const d2*>(E + off);
                        if constexpr (FE) e = csub(e, cscale(*reinterpret_cast<const d2*>(E2 + off), 1.0 / rs[j].mu));
                        v = MODE == 1 ? make_double2(e.x - v.x, e.y - v.y) : make_double2(e.x + v.x, e.y + v.y);
                    }
                    *reinterpret_cast<d2*>(C + off) = v;
                }
            }
}
}  // namespace

template <class CF>
void launch_zgemm3m_cfg(int mode, bool conj_l, int M, int K, int nb, const double* L, int ldl, long long strideL,
                        const double* V, int ldv, long long strideV, double* C, const double* E, int ldc,
                        long long strideC, int nz, hipStream_t st, const double* klim = nullptr,
                        long long klim_stride = 0) {
    const int tilesI = (M + CF::BC - 1) / CF::BC;
    const int tilesJ = (nb + CF::BJ - 1) / CF::BJ;
    dim3 grid(tilesI * tilesJ, 1, nz), block(CF::NT);
#define ACE_GEMM_LAUNCH(MD, CJ)                                                                                    \
    hipLaunchKernelGGL((zgemm3m_kernel<MD, CJ, CF>), grid, block, 0, st, M, K, nb, L, ldl, strideL, V, ldv, strideV, \
                       C, E, ldc, strideC, tilesI, tilesJ, nullptr, nullptr, nullptr, YsArgs{}, klim, klim_stride)
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

// Launch one GEMM with tile configuration CF (also used by tools/probe_gemm.hip).
template <class CF>
void launch_zgemm_cfg(int mode, bool conj_l, int M, int K, int nb, const double* L, int ldl, long long strideL,
                      const double* V, int ldv, long long strideV, double* C, const double* E, int ldc,
                      long long strideC, int nz, hipStream_t st) {
    const int tilesI = (M + CF::BI / 2 - 1) / (CF::BI / 2);
    const int tilesJ = (nb + CF::BJ - 1) / CF::BJ;
    dim3 grid(tilesI * tilesJ, 1, nz), block(CF::NT);
#define ACE_GEMM_LAUNCH(MD, CJ)                                                                                  \
    hipLaunchKernelGGL((zgemm_kernel<MD, CJ, CF>), grid, block, 0, st, M, K, nb, L, ldl, strideL, V, ldv, strideV, \
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

void launch_zgemm(int mode, bool conj_l, int M, int K, int nb, const double* L, int ldl, long long strideL,
                  const double* V, int ldv, long long strideV, double* C, const double* E, int ldc,
                  long long strideC, int nz, hipStream_t st, const double* klim, long long klim_stride) {
    // 3M kernel (measured on MI355X, tools/probe_gemm.hip, unit shapes: apply_A 196 -> 135 us, apply_AH
    // 194 -> 135 us, G/K 52.6 -> 38.4 us against the 4M GemmDefault).  8 waves per work-group; the
    // 64 x 32 output tile when the 64 x 64 one would leave fewer than 512 work-groups.
    using Big = Gemm3mCfg<64, 64, 16, 2, 4>;
    using Small = Gemm3mCfg<64, 32, 16, 4, 2>;
    const long long big_blocks = (long long)((M + 63) / 64) * ((nb + 63) / 64) * nz;
    if (big_blocks >= 256 && M >= 64)
        launch_zgemm3m_cfg<Big>(mode, conj_l, M, K, nb, L, ldl, strideL, V, ldv, strideV, C, E, ldc, strideC, nz, st,
                                klim, klim_stride);
    else
        launch_zgemm3m_cfg<Small>(mode, conj_l, M, K, nb, L, ldl, strideL, V, ldv, strideV, C, E, ldc, strideC, nz, st,
                                  klim, klim_stride);
}

// g = G T with the Y-step in the epilogue (r = 1, shared G).  ys.part: [nb][ceil(m/64)][5].
void launch_zgemm_ystep(int m, int nb, const double* G, const double* T, double* g, const YsArgs& ys,
                        const RealState* rs, hipStream_t st) {
    using CF = Gemm3mCfg<64, 64, 16, 2, 4>;
    const int tilesI = (m + CF::BC - 1) / CF::BC;
    const int tilesJ = (nb + CF::BJ - 1) / CF::BJ;
    dim3 grid(tilesI * tilesJ, 1, 1), block(CF::NT);
    hipLaunchKernelGGL((zgemm3m_kernel<0, false, CF, false, false, true>), grid, block, 0, st, m, m, nb, G, m, 0LL, T,
                       m, 0LL, g, nullptr, m, 0LL, tilesI, tilesJ, nullptr, nullptr, rs, ys);
}

// Shared-A products of the r = 1 iteration with pre_kernel folded in (Big tile configuration):
//   apply_A  (fv):  C = (E - E2/mu) - A (V - V2/mu)       T = S - A V  with S = Y - M/mu, V = Z - N/mu
//   apply_AH (!fv): C = (E - E2/mu) + A^H V               X = V + A^H g with V = Z - N/mu
void launch_zgemm_fused(bool fv, int M, int K, int nb, const double* L, int ldl, const double* V, const double* V2,
                        int ldv, double* C, const double* E, const double* E2, int ldc, const RealState* rs,
                        hipStream_t st) {
    using CF = Gemm3mCfg<64, 64, 16, 2, 4>;
    const int tilesI = (M + CF::BC - 1) / CF::BC;
    const int tilesJ = (nb + CF::BJ - 1) / CF::BJ;
    dim3 grid(tilesI * tilesJ, 1, 1), block(CF::NT);
    if (fv)
        hipLaunchKernelGGL((zgemm3m_kernel<1, false, CF, true, true>), grid, block, 0, st, M, K, nb, L, ldl, 0LL, V,
                           ldv, 0LL, C, E, ldc, 0LL, tilesI, tilesJ, V2, E2, rs);
    else
        hipLaunchKernelGGL((zgemm3m_kernel<2, false, CF, false, true>), grid, block, 0, st, M, K, nb, L, ldl, 0LL, V,
                           ldv, 0LL, C, E, ldc, 0LL, tilesI, tilesJ, V2, E2, rs);
}

}  // namespace ace
