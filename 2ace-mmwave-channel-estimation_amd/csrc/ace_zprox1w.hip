// A2only Z-step, one wave per realisation (inferLowRankV4_multi.m:423-485 with the
// residual / stopping / mu logic of :340-382).
//
// Layout of one realisation on its wave:
//   LDS  T0: one 32x33 complex tile (16.9 KiB) -- E, F, the packed double-buffered
//        Hermitian matrix during the sweeps, R / Qnew afterwards.  With ~17 KiB per
//        wave the CU keeps every realisation of a 4096-batch resident at once.
//   VGPR R : the accumulated Jacobi rotations in the position frame: lane (g, k) =
//        (lane >> 4, lane & 15) holds R[i][2k], R[i][2k+1] for rows i = g + 4r.  The
//        circle-method position permutation after each step is a one-lane shift
//        inside each 16-lane DPP row (row_shr:1 / row_shl:1).
// Products (all on v_mfma_f64_16x16x4_f64, 16x16 complex output blocks):
//   warm  F = Qprev^H E,   H = F F^H   (= Qprev^H E E^H Qprev: nearly diagonal)
//   cold  H = E E^H
//   post  Qnew = Qprev R,  T = diag(sqrt(scale)) Qnew^H E,  Z^T = T^T Qnew^T
// where the accumulator of T is used directly as the A operand of the last product
// (the f64 MFMA accumulator row map (l>>4)+4q equals the operand k map), and Z^T
// puts consecutive vec(Z) indices on consecutive lanes for coalesced stores.
#include "ace_common.hpp"
#include "ace_zcommon.hpp"
#include "ace_topk.hpp"

namespace ace {

namespace {

__device__ __forceinline__ double dpp_shr1(double x) {  // lane k <- lane k-1 within each 16-lane row
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x111, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x111, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_shl1(double x) {  // lane k <- lane k+1 within each 16-lane row
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x101, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x101, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
// The same shifts with the row-end lane keeping `old` (it has no source lane and bound_ctrl is off):
// row_shr:1 leaves lane 0 of each row with old, row_shl:1 lane 15.  One DPP move per dword, no select.
__device__ __forceinline__ double dpp_shr1_keep(double old, double x) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(x), 0x111, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(x), 0x111, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_shl1_keep(double old, double x) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(x), 0x101, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(x), 0x101, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ void mfma_c(d2 a, d2 b, d4v& cr, d4v& ci) {  // (cr, ci) += a * b (complex)
    cr = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, b.x, cr, 0, 0, 0);
    cr = __builtin_amdgcn_mfma_f64_16x16x4f64(-a.y, b.y, cr, 0, 0, 0);
    ci = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, b.y, ci, 0, 0, 0);
    ci = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, b.x, ci, 0, 0, 0);
}

// 16x16 complex block C = sum_k A[row][k] B[k][col] over k < 32.  fa(row, k) and
// fb(k0, k, col) return operand values for this lane (row/col in 0..15 within the
// block, k the absolute inner index; k0 the 4-aligned step base, compile-time after
// unrolling, for register-resident operands).
template <class FA, class FB>
__device__ __forceinline__ void mm16(FA fa, FB fb, d4v& cr, d4v& ci, int lane) {
    cr = d4v{0.0, 0.0, 0.0, 0.0};
    ci = d4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k0 = 0; k0 < 32; k0 += 4) {
        const int kk = k0 + (lane >> 4);
        mfma_c(fa(lane & 15, kk), fb(k0, kk, lane & 15), cr, ci);
    }
}

// off-diagonal 16x16 slot-pair blocks (ka < kb) for the one-wave sweep: two per lane; the 16 diagonal
// blocks are updated by the lanes that form their pair's rotation (zstep1w_body)
static __constant__ unsigned char c_off_a[120] = {0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,1,1,1,1,1,1,1,1,1,1,1,1,1,1,2,2,2,2,2,2,2,2,2,2,2,2,2,3,3,3,3,3,3,3,3,3,3,3,3,4,4,4,4,4,4,4,4,4,4,4,5,5,5,5,5,5,5,5,5,5,6,6,6,6,6,6,6,6,6,7,7,7,7,7,7,7,7,8,8,8,8,8,8,8,9,9,9,9,9,9,10,10,10,10,10,11,11,11,11,12,12,12,13,13,14};
static __constant__ unsigned char c_off_b[120] = {1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,2,3,4,5,6,7,8,9,10,11,12,13,14,15,3,4,5,6,7,8,9,10,11,12,13,14,15,4,5,6,7,8,9,10,11,12,13,14,15,5,6,7,8,9,10,11,12,13,14,15,6,7,8,9,10,11,12,13,14,15,7,8,9,10,11,12,13,14,15,8,9,10,11,12,13,14,15,9,10,11,12,13,14,15,10,11,12,13,14,15,11,12,13,14,15,12,13,14,15,13,14,15,14,15,15};

// m-space fallback (RealState::msp): the bound failed for an iterate gyk_kernel settled in m-space,
// so the full Z-step needs Z and X = Z' in memory.  One wave forms them from the implicit form,
// out = base + A^H v with the f64 A (rare: the bound keeps holding once it holds), and opt_X if
// it lives in m-space form or in a Z buffer about to be rewritten.
__device__ __forceinline__ void msp_materialise(const ZArgs& a, int b) {
    const int lane = threadIdx.x, n = a.n, m = a.m;
    RealState* st = a.st + b;
    const int zc_id = (a.it & 1) ? 1 : 2, zn_id = 1 + (a.it & 1);
    const int z0id = st->z0id, optsrc = st->optsrc, entered = st->msp_pad == a.it;
    d2* Zc = reinterpret_cast<d2*>(a.Z) + (long long)b * n;
    d2* Zn = reinterpret_cast<d2*>(a.Zn) + (long long)b * n;
    d2* Z0 = z0id == zc_id ? Zc : Zn;
    d2* oX = reinterpret_cast<d2*>(a.optX) + (long long)b * n;
    const d2* Af = reinterpret_cast<const d2*>(a.Af);
    const long long om = (long long)b * m;
    auto gemv = [&](d2* out, const d2* base, const d2* v) {   // out[k] = base[k] + sum_i conj(A[i][k]) v[i]
        for (int k0 = 0; k0 < n; k0 += 64 * 4) {
            d2 acc[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[u] = make_double2(0.0, 0.0);
            for (int i = 0; i < m; ++i) {
                const d2 vi = v[i];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = min(k0 + lane + 64 * u, n - 1);
                    const d2 av = Af[(long long)i * n + k];
                    acc[u].x = fma(av.x, vi.x, fma(av.y, vi.y, acc[u].x));
                    acc[u].y = fma(av.x, vi.y, fma(-av.y, vi.x, acc[u].y));
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + lane + 64 * u;
                if (k < n) out[k] = cadd(base[k], acc[u]);
            }
        }
        __syncthreads();   // (one wave) the stores are visible to every lane's later loads
    };
    if (optsrc >= 3 && optsrc <= 5) {   // opt_S, or still in the S buffer Sg[optsrc - 4]
        const double* sp = optsrc == 3 ? a.optS : ((optsrc - 4) == (a.it & 1) ? a.Snew : a.Sold);
        gemv(oX, Z0, reinterpret_cast<const d2*>(sp) + om);
    } else if (optsrc == zc_id || optsrc == zn_id) {
        const d2* src = optsrc == zc_id ? Zc : Zn;
        for (int k = lane; k < n; k += 64) oX[k] = src[k];
        __syncthreads();
    }
    const d2* Sn = reinterpret_cast<const d2*>(a.Snew) + om;
    const d2* So = reinterpret_cast<const d2*>(a.Sold) + om;
    if (Z0 == Zc) {
        gemv(Zn, Zc, Sn);
        if (!entered) gemv(Zc, Zc, So);
    } else {
        gemv(Zc, Zn, So);   // (entered implies Z0 == Zc)
        gemv(Zn, Zn, Sn);
    }
    if (lane == 0) {
        if ((optsrc >= 3 && optsrc <= 5) || optsrc == zc_id || optsrc == zn_id) st->optsrc = 0;
        st->msp = 0;
    }
    __syncthreads();
}

// ---- rank-one profile: the top eigenpair only --------------------------------------------------
// With the profile [1] / [0.95] (use_rank_one, inferLowRankV4_multi.m:448-450) the tail rescaling
// (:469-480) multiplies every eigenvalue but the largest by one factor c = min(1, vr / (v - vr) (1/f - 1)),
// vr = lambda_1, v = the eigenvalue sum, so Z = U diag(sqrt(scale)) U^H E (:482-484) needs only
// (lambda_1, u_1): Z = sqrt(c) E + (1 - sqrt(c)) u_1 u_1^H E.  r1_top finds them with Lanczos (full
// reorthogonalisation) on the packed H = F F^H of the warm frame, started at the unit vector of H's
// largest diagonal entry (column 0 of the warm start Q_prev holds the previous u_1: nearly converged),
// and certifies the result: the Ritz residual beta_k |s_k| <= 2^-48 theta, and theta the LARGEST
// eigenvalue (theta > v - theta, or sigma I - H positive definite for sigma just above theta: a
// Cholesky).  Anything else returns false and the caller runs the full Jacobi eigensolver.
constexpr int LZ_MAX = 16;   // Lanczos steps before giving up (the Jacobi path then runs)

__device__ __forceinline__ double half_sum(double v) {   // sum over lanes 0..31 (both halves hold it)
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// largest eigenvalue and its eigenvector of the symmetric tridiagonal T (diag al[0..k), off be[1..k):
// be[j] couples j - 1 and j), all in LDS: 64-lane multisection on Sturm counts, then on lane 0 the twisted
// factorisation (LAPACK dlar1v) for the vector s[0..k) (normalised, in LDS; dp, dm: LDS scratch)
__device__ __forceinline__ double tri_top(const double* al, const double* be, int k, int lane, double* s, double* dp,
                                       double* dm) {
    double lo = al[0], hi = al[0];
    for (int j = 0; j < k; ++j) {
        const double r = (j > 0 ? fabs(be[j]) : 0.0) + (j + 1 < k ? fabs(be[j + 1]) : 0.0);
        lo = fmin(lo, al[j] - r);
        hi = fmax(hi, al[j] + r);
    }
    const double scale = fmax(fabs(lo), fabs(hi));
    const double tiny = 1e-300 + 1e-30 * scale * 2.2e-16;
    for (int round = 0; round < 12 && hi - lo > 2.2e-16 * scale; ++round) {
        const double x = lo + (hi - lo) * (double)(lane + 1) / 65.0;
        int neg = 0;   // Sturm count: eigenvalues < x
        double d = al[0] - x;
        if (d == 0.0) d = -tiny;
        neg += d < 0.0;
        for (int j = 1; j < k; ++j) {
            d = (al[j] - x) - be[j] * be[j] / d;
            if (d == 0.0) d = -tiny;
            neg += d < 0.0;
        }
        const int above = k - neg;
        // the top eigenvalue lies in (x_i, x_{i+1}] with count(x_i) >= 1 > count(x_{i+1}) = 0
        double nlo = above >= 1 ? x : lo, nhi = above == 0 ? x : hi;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            nlo = fmax(nlo, __shfl_xor(nlo, o, 64));
            nhi = fmin(nhi, __shfl_xor(nhi, o, 64));
        }
        lo = nlo;
        hi = nhi;
    }
    const double th = 0.5 * (lo + hi);
    if (lane == 0) {   // twisted factorisation at th
        for (int j = 0; j < k; ++j) {
            const double d = (al[j] - th) - (j > 0 ? be[j] * be[j] / dp[j - 1] : 0.0);
            dp[j] = d == 0.0 ? tiny : d;
        }
        for (int j = k - 1; j >= 0; --j) {
            const double d = (al[j] - th) - (j + 1 < k ? be[j + 1] * be[j + 1] / dm[j + 1] : 0.0);
            dm[j] = d == 0.0 ? tiny : d;
        }
        int r = 0;
        double gbest = INFINITY;
        for (int j = 0; j < k; ++j) {
            const double g = fabs(dp[j] + dm[j] - (al[j] - th));
            if (g < gbest) { gbest = g; r = j; }
        }
        s[r] = 1.0;
        double nrm = 1.0;
        for (int j = r - 1; j >= 0; --j) { s[j] = -be[j + 1] * s[j + 1] / dp[j]; nrm += s[j] * s[j]; }
        for (int j = r + 1; j < k; ++j) { s[j] = -be[j] * s[j - 1] / dm[j]; nrm += s[j] * s[j]; }
        const double inv = 1.0 / sqrt(nrm);
        for (int j = 0; j < k; ++j) s[j] *= inv;
    }
    __syncthreads();
    return th;
}

// H: packed upper Hermitian (up_idx), zero beyond tx; Vb: LDS scratch of ZPACK complex (the Lanczos basis,
// LZ_MAX x 32, then the Cholesky copy); tri: LDS scratch of 5 LZ_MAX + 2 doubles.  On success y (component
// lane & 31 of the unit top eigenvector) and theta.
__device__ __forceinline__ bool r1_top(const d2* H, d2* Vb, double* tri, int tx, int lane, double tr, d2& y, double& theta) {
    const int i = lane & 31, h = lane >> 5;
    double* al = tri;                     // alpha_0 ..
    double* be = tri + LZ_MAX;            // beta_1 .. at be[1 ..]
    double* sv = tri + 2 * LZ_MAX + 1;    // Ritz vector of T
    double* dp = sv + LZ_MAX;
    double* dm = dp + LZ_MAX;
    if (!(tr > 0.0)) return false;
    // start: the unit vector of the largest diagonal entry (first index on ties)
    double dg = i < tx ? H[up_idx(i, i)].x : -1.0;
    int i0 = i;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
        const double od = __shfl_xor(dg, o, 64);
        const int oi = __shfl_xor(i0, o, 64);
        if (od > dg || (od == dg && oi < i0)) { dg = od; i0 = oi; }
    }
    d2 q = make_double2(i == i0 ? 1.0 : 0.0, 0.0), qprev = make_double2(0.0, 0.0);
    double bk = 0.0;   // beta_k
    bool conv = false;
    int k = 0;
    for (; k < LZ_MAX && k < tx; ++k) {
        if (h == 0) Vb[k * 32 + i] = q;
        __syncthreads();
        // w = H q_k: row i, columns 16h .. 16h + 15, then the two halves combined
        double wr = 0.0, wi = 0.0;
        for (int c = 16 * h; c < 16 * h + 16; ++c) {
            const d2 hv = i <= c ? H[up_idx(i, c)] : conj_d2(H[up_idx(c, i)]), v = Vb[k * 32 + c];
            wr += hv.x * v.x - hv.y * v.y;
            wi += hv.x * v.y + hv.y * v.x;
        }
        wr = xor32_sum(wr);
        wi = xor32_sum(wi);
        const double alpha = half_sum(q.x * wr + q.y * wi);   // Re q^H w
        wr -= alpha * q.x + bk * qprev.x;
        wi -= alpha * q.y + bk * qprev.y;
        for (int pass = 0; pass < 2; ++pass)                  // full reorthogonalisation, twice
            for (int j = 0; j <= k; ++j) {
                const d2 v = Vb[j * 32 + i];
                const double cr = half_sum(v.x * wr + v.y * wi), ci = half_sum(v.x * wi - v.y * wr);
                wr -= cr * v.x - ci * v.y;
                wi -= cr * v.y + ci * v.x;
            }
        const double bn = sqrt(half_sum(wr * wr + wi * wi));
        if (lane == 0) {
            al[k] = alpha;
            be[k + 1] = bn;
        }
        __syncthreads();
        const int kk = k + 1;
        const bool inv = !(bn > 1e-300 * tr);   // an invariant subspace: the Ritz values are exact
        if (kk % 4 == 0 || kk == tx || kk == LZ_MAX || inv) {
            theta = tri_top(al, be, kk, lane, sv, dp, dm);
            if (inv || kk == tx || bn * fabs(sv[kk - 1]) <= 0x1p-48 * theta) {
                conv = theta > 0.0;
                k = kk;
                break;
            }
        }
        qprev = q;
        q = make_double2(wr / bn, wi / bn);
        bk = bn;
    }
    if (!conv) return false;
    // Ritz vector y = V s
    double yr = 0.0, yi = 0.0;
    for (int j = 0; j < k; ++j) {
        const d2 v = Vb[j * 32 + i];
        yr += sv[j] * v.x;
        yi += sv[j] * v.y;
    }
    const double yn = 1.0 / sqrt(half_sum(yr * yr + yi * yi));
    y = make_double2(yr * yn, yi * yn);
    // theta is the largest eigenvalue: every other is <= tr - theta < theta, or sigma I - H > 0
    if (theta > 0.5 * tr * (1.0 + 1e-12)) return true;
    const double sigma = theta * (1.0 + 1e-11);
    __syncthreads();
    d2* C = Vb;   // packed copy of sigma I - H
    for (int e = lane; e < ZPACK; e += 64) {
        const d2 v = H[e];
        C[e] = make_double2(-v.x, -v.y);
    }
    __syncthreads();
    if (lane < 32) C[up_idx(lane, lane)].x += sigma;
    __syncthreads();
    int bad = 0;
    for (int c = 0; c < tx; ++c) {   // right-looking Cholesky: row c of U, then the trailing rows
        const double d = C[up_idx(c, c)].x;
        if (!(d > 0.0)) { bad = 1; break; }
        const double is = 1.0 / sqrt(d);
        __syncthreads();
        for (int j = c + 1 + lane; j < tx; j += 64) C[up_idx(c, j)] = cscale(C[up_idx(c, j)], is);
        __syncthreads();
        for (int r2 = c + 1 + i; r2 < tx; r2 += 32)
            for (int j = r2 + h; j < tx; j += 2) {
                const d2 ur = C[up_idx(c, r2)], uj = C[up_idx(c, j)];
                // A_rj -= conj(U_cr) U_cj
                C[up_idx(r2, j)] = csub(C[up_idx(r2, j)], make_double2(ur.x * uj.x + ur.y * uj.y, ur.x * uj.y - ur.y * uj.x));
            }
        __syncthreads();
    }
    return !bad;
}

template <bool INIT>
__device__ __forceinline__ void zstep1w_body(const ZArgs& a, int b) {
    const int lane = threadIdx.x;
    const int n = a.n, m = a.m, tx = a.tx, rx = a.rx;
    RealState* st = a.st + b;
    // the three state words the steady state decides on, requested together (one round trip
    // instead of a chain of dependent loads before the common early exits)
    // (the empty asm consumes all of them before the first branch, so that the compiler cannot
    // sink each load below the branch before it: one memory round trip, not four)
    int s_done = 0, s_zit = 0, s_fzit = 0;
    if (!INIT) {
        s_done = st->done;
        s_zit = st->zit;
        s_fzit = st->fzit;
    }
    const int r1 = a.rank_one ? (int)a.rank_one[b] : 0;
    asm volatile("" ::"s"(s_done), "s"(s_zit), "s"(s_fzit), "v"(r1));
    const ZProfile pf = z_profile_flag(a, r1);
    if (!INIT && s_done) return;
    // zlean_kernel or the fused control completed this iteration (msr_kernel: this and later ones)
    if (!INIT && a.lean && s_zit >= a.it) return;
    // The fused apply_AH formed X = Z + W of this iteration in Z' with its sums: the perturbation
    // certificate of zlean_kernel, then the iteration control; if the bound fails, the full
    // Z-step below runs on X read from Z'.
    const bool xin = !INIT && a.xfuse && s_fzit == a.it;
    if (xin) {
        int ok = 0;
        if (threadIdx.x == 0) ok = fused_control(a, st, pf);
        ok = __shfl(ok, 0, 64);
        if (ok) {
            if ((ok & 2) && a.fixup_now) dual_fixup(a, b, st);   // pending test at the last iteration
            return;
        }
        if (a.msp && st->mzit == a.it) msp_materialise(a, b);
    }
    __shared__ __attribute__((aligned(16))) d2 T0[ZT * ZHS];
    __shared__ double4 RotS[16];
    __shared__ double wv[ZT], scl[ZT], rs2[ZT];
    __shared__ int ord[ZT], ascp[ZT];
    __shared__ int flag_any, flag_fast;
    __shared__ double lz_tri[5 * LZ_MAX + 2];   // r1_top's tridiagonal and scratch

    const double mu = INIT ? 1.0 : st->mu;
    const d2* X = reinterpret_cast<const d2*>(xin ? a.Zn : a.X) + (long long)b * n;
    // wmode + ping-pong: N may be the exact zero vector (RealState::nzero), and in the common case
    // Z = E the new N is stored as exact zero (see RealState::nzero)
    const bool flushN = !INIT && a.wmode && a.Zn && a.Zn != a.Z && a.zeros;
    const bool nz_in = flushN && st->nzero;
    const d2* N = nz_in ? reinterpret_cast<const d2*>(a.zeros) : reinterpret_cast<const d2*>(a.N) + (long long)b * n;
    const d2* Z = reinterpret_cast<const d2*>(a.Z) + (long long)b * n;
    d2* Nn = reinterpret_cast<d2*>(a.Nn ? a.Nn : a.N) + (long long)b * n;
    d2* Zn = reinterpret_cast<d2*>(a.Zn ? a.Zn : a.Z) + (long long)b * n;
    const bool pp = !INIT && a.Zn && a.Zn != a.Z && a.Nn != a.N;   // ping-pong outputs
    d2* Qg = reinterpret_cast<d2*>(a.Q) + (long long)b * tx * tx;
    const bool nuc = a.nuclear;   // inferLowRank_Nuclear.m:411-419 at r = 1 (no eigendecomposition)
    const bool warm = (!INIT) && a.warm && !nuc;
    const double imu = 1.0 / mu;
    // wmode: the X buffer holds W = A^H g and X = (Z - N/mu) + W is formed here
    const bool wm = !INIT && a.wmode && !xin;
    auto loadx = [&](int k, d2 nn, d2 zo) -> d2 {
        const d2 v = X[k];
        return wm ? xw(zo, nn, v, imu) : v;
    };
    auto evalE = [&](int k) -> d2 {  // X + N/mu (:424), as N * (1/mu) like pre_kernel's V = Z - N/mu
        const d2 nn = N[k];
        const d2 x = loadx(k, nn, wm ? Z[k] : nn);
        return make_double2(fma(nn.x, imu, x.x), fma(nn.y, imu, x.y));
    };
    const d2 zero = make_double2(0.0, 0.0);
    // Whether this iterate becomes opt_X (:344-351) depends only on the Y-step's objective, so
    // it is decided up front and X is copied as it is formed (iter_control makes the same decision).
    double obj2_now = 0.0;
    if (!INIT) {
        if (a.ypart) {
            double v[5];
            ystep_sums(a, b, v);
            obj2_now = v[0];
        } else {
            obj2_now = st->obj2;
        }
    }
    const bool improved_pre = !INIT && sqrt(obj2_now) < st->opt_obj;
    const bool keep_cur = wm && !improved_pre && !(st->opt_obj < INFINITY);   // finalize's fallback X
    d2* oX = reinterpret_cast<d2*>(a.optX) + (long long)b * n;
    d2* Xc = reinterpret_cast<d2*>(a.Xcur) + (long long)b * n;
    // Deferred opt_X (RealState::optsrc): with N = 0 and Z = E the new Z' equals X exactly, so an
    // improved iterate is only recorded as "in the Z' buffer"; it is copied to opt_X when that
    // buffer is about to be overwritten (here, two iterations later) if no better iterate came.
    const int zn_id = 1 + (a.it & 1);   // Z' buffer of this iteration: Z2 for odd it, Z for even
    int optsrc = INIT ? 0 : st->optsrc;
    if (pp && optsrc == zn_id) {
        for (int k = lane; k < n; k += 64 * 4) {   // four loads in flight, named (no local array)
            const d2 v0 = Zn[k], v1 = Zn[min(k + 64, n - 1)], v2 = Zn[min(k + 128, n - 1)],
                     v3 = Zn[min(k + 192, n - 1)];
            oX[k] = v0;
            if (k + 64 < n) oX[k + 64] = v1;
            if (k + 128 < n) oX[k + 128] = v2;
            if (k + 192 < n) oX[k + 192] = v3;
        }
        optsrc = 0;
    }
    const bool defer_opt = improved_pre && nz_in && pp;   // decided after the certificate
    // m-space dual terms ||A^H (Y - Y0)||^2 = dY^H (K Y - K Y0), ||A^H Y||^2 = Y^H K Y, and opt_Y:
    // they depend only on the Y-step and K Y, so they run first (their loads then do not queue
    // behind this kernel's stores)
    double dAtY = 0.0, nAtY = 0.0;
    if (!INIT && a.yfused) {   // gyk_kernel produced the dual terms and opt_Y
        if (lane == 0) {
            dAtY = st->dAtY;
            nAtY = st->nAtY;
        }
    } else if (!INIT) {
        const d2* Yn = reinterpret_cast<const d2*>(a.Ynew) + (long long)b * m;
        const d2* Yo = reinterpret_cast<const d2*>(a.Yold) + (long long)b * m;
        const d2* Kn = reinterpret_cast<const d2*>(a.KYnew) + (long long)b * m;
        const d2* Ko = reinterpret_cast<const d2*>(a.KYold) + (long long)b * m;
        d2* oY = reinterpret_cast<d2*>(a.optY) + (long long)b * m;
        auto term = [&](int i, d2 yn, d2 yo, d2 kn, d2 ko) {
            const d2 dy = csub(yn, yo), dk = csub(kn, ko);
            dAtY += dy.x * dk.x + dy.y * dk.y;
            nAtY += yn.x * kn.x + yn.y * kn.y;
            if (improved_pre) oY[i] = yn;   // best-objective iterate (:344-351; iter_control agrees)
        };
        constexpr int YS = 4;   // the first 4 x 64 entries with all loads in flight at once
        d2 yn[YS], yo[YS], kn[YS], ko[YS];
#pragma unroll
        for (int q = 0; q < YS; ++q) {
            const int i = lane + 64 * q, ic = i < m ? i : 0;
            yn[q] = Yn[ic];
            yo[q] = Yo[ic];
            kn[q] = Kn[ic];
            ko[q] = Ko[ic];
        }
#pragma unroll
        for (int q = 0; q < YS; ++q)
            if (lane + 64 * q < m) term(lane + 64 * q, yn[q], yo[q], kn[q], ko[q]);
        for (int i = lane + 64 * YS; i < m; i += 64) term(i, Yn[i], Yo[i], Kn[i], Ko[i]);
    }
#ifdef ACE_DEBUG_SWEEPS
    const unsigned long long dbg_t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long dbg_t1 = dbg_t0, dbg_t2 = dbg_t0, dbg_t3 = dbg_t0, dbg_fa = 0, dbg_fb = 0, dbg_fc = 0;
    int sweeps = -1;
#else
    int sweeps = 0;
#endif

    // Qprev operand fragments of the warm product F = Qprev^H E, fetched first so that their
    // latency overlaps the E loads: qv[I][s] = Qprev[4s + (lane>>4)][16I + (lane&15)] (identity
    // padded).  Qprev's columns are stored in descending eigenvalue order (below), so when every
    // profile rank is <= 16 the certificate needs only F's first 16 rows (I = 0); the second
    // half is fetched only if the certificate fails.
    int maxr = 0;
    #pragma unroll
    for (int pi = 0; pi < 4; ++pi) maxr = pi < pf.np ? max(maxr, pf.rl[pi]) : maxr;
    const bool top16 = warm && maxr <= 16;
    d2 qv[2][8];
    auto load_q = [&](int I) {
#pragma unroll
        for (int s8 = 0; s8 < 8; ++s8) {
            const int i = 4 * s8 + (lane >> 4), k = 16 * I + (lane & 15);
            qv[I][s8] = (i < tx && k < tx) ? Qg[i * tx + k] : make_double2(i == k ? 1.0 : 0.0, 0.0);
        }
    };
    if (warm) {
        load_q(0);
        if (!top16) load_q(1);
    }
    // ---- E = reshape(X + N/mu, tx, []) (:424-426), zero padded to 32x32.  Loads are issued
    // in chunks of 8 per lane ahead of the LDS stores (memory-level parallelism).
    // Speculative outputs of the common case Z = E (no tail rescaling): N' = N + mu (X - E) and
    // the four sums, kept in registers until the certificate decides (element e = lane + 64 u).
    double etr = 0.0;  // ||E||_F^2 = trace(E E^H)
    double sacc[4] = {0.0, 0.0, 0.0, 0.0};
    VMax svz, svn;
    // Four chunks of 4 elements per lane, the loads of chunk c + 1 issued before the stores of
    // chunk c (vmcnt retires in order: loads queued behind stores would wait for them); the
    // loads are unconditional (clamped index, zeroed outside the tx x rx block).
    struct Ch {
        d2 x[4], n[4], z[4];
    };
    auto cload = [&](int c, Ch& q) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = lane + 64 * (4 * c + u), i = e & 31, j = e >> 5;
            const int k = (i < tx && j < rx) ? i + tx * j : 0;
            q.x[u] = X[k];
            q.n[u] = N[k];
            q.z[u] = INIT ? zero : Z[k];
        }
    };
    auto cwork = [&](int c, const Ch& q) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = lane + 64 * (4 * c + u), i = e & 31, j = e >> 5, k = i + tx * j;
            const bool in = i < tx && j < rx;
            const d2 xv = in ? q.x[u] : zero, nv = in ? q.n[u] : zero, zv = in ? q.z[u] : zero;
            const d2 x = wm ? xw(zv, nv, xv, imu) : xv;
            const d2 ev = in ? make_double2(fma(nv.x, imu, x.x), fma(nv.y, imu, x.y)) : zero;
            etr += cabs2(ev);
            T0[i * ZHS + j] = ev;
            if (in && !INIT) {
                if (improved_pre && !defer_opt) oX[k] = x;
                else if (keep_cur) Xc[k] = x;
                const d2 d = csub(x, ev);
                const d2 nn = cadd(nv, cscale(d, mu));
                if (pp) {
                    Zn[k] = ev;
                    if (!flushN) Nn[k] = nn;
                }
                sacc[0] += cabs2(x);
                sacc[1] += cabs2(ev);
                sacc[2] += cabs2(d);
                sacc[3] += cabs2(csub(ev, zv));
                svz.add(ev);
                svn.add(nn);
            }
        }
    };
    {
        Ch c0, c1;
        cload(0, c0);
        cload(1, c1);
        cwork(0, c0);
        cload(2, c0);
        cwork(1, c1);
        cload(3, c1);
        cwork(2, c0);
        cwork(3, c1);
    }
    __syncthreads();
#ifdef ACE_DEBUG_SWEEPS
    dbg_fa = __builtin_amdgcn_s_memrealtime();
#endif
    // Qprev with identity padding
    auto qprev = [&](int i, int k) -> d2 {
        if (i < tx && k < tx) return Qg[i * tx + k];
        return make_double2(i == k ? 1.0 : 0.0, 0.0);
    };
    d4v cr[2][2], ci[2][2];
    auto warm_half = [&](int I) {  // rows 16I..16I+15 of F = Qprev^H E (T0 = E)
#pragma unroll
        for (int J = 0; J < 2; ++J) {
            cr[I][J] = d4v{0.0, 0.0, 0.0, 0.0};
            ci[I][J] = d4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s8 = 0; s8 < 8; ++s8) {
                const d2 q = qv[I][s8];
                mfma_c(make_double2(q.x, -q.y), T0[(4 * s8 + (lane >> 4)) * ZHS + 16 * J + (lane & 15)], cr[I][J],
                       ci[I][J]);
            }
        }
    };
    auto store_f = [&]() {  // T0 = F (after every wave has finished reading E)
        __syncthreads();
#pragma unroll
        for (int I = 0; I < 2; ++I)
#pragma unroll
            for (int J = 0; J < 2; ++J)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    T0[(16 * I + (lane >> 4) + 4 * r) * ZHS + 16 * J + (lane & 15)] =
                        make_double2(cr[I][J][r], ci[I][J][r]);
        __syncthreads();
    };
    if (warm) {
        warm_half(0);
        if (!top16) warm_half(1);
    }
#ifdef ACE_DEBUG_SWEEPS
    dbg_fb = __builtin_amdgcn_s_memrealtime();
#endif
    // ---- Spectral certificate.  The tail rescaling (:469-480) fires only when some
    // profile entry has  sum(top-r eigenvalues) < f * trace.  By Ky Fan, the sum of the r
    // largest diagonal entries of Q^H H Q (= squared row norms of F = Q^H E) is a lower bound
    // on sum(top-r eigenvalues) for any Q with orthonormal columns, and trace(H) = ||E||_F^2.
    // When every entry clears its threshold by a relative margin far above the rounding of
    // the reference's eig, no rescaling happens there either and Z = E exactly: the
    // eigendecomposition is skipped (Q keeps its warm start).
    bool fast_reg = false;
    double kfv[4] = {0.0, 0.0, 0.0, 0.0};   // sqrt of the certified top-r row sums (RealState::kf)
    if (!INIT && top16) {
        // row norms of F's first 16 rows straight from the accumulators: lane l holds rows
        // (l>>4) + 4r, columns l&15 (+16J); reduce over the 16 column lanes
        double rn[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            double v = 0.0;
#pragma unroll
            for (int J = 0; J < 2; ++J) v += cr[0][J][r] * cr[0][J][r] + ci[0][J][r] * ci[0][J][r];
            rn[r] = bsum16(v);
        }
        // lane L (of each 16-lane group) takes row L = (L&3) + 4(L>>2)
        const int L16 = lane & 15;
        double t0 = __shfl(rn[0], 16 * (L16 & 3), 64), t1 = __shfl(rn[1], 16 * (L16 & 3), 64);
        double t2 = __shfl(rn[2], 16 * (L16 & 3), 64), t3 = __shfl(rn[3], 16 * (L16 & 3), 64);
        const int rsel = L16 >> 2;
        double val = rsel == 0 ? t0 : (rsel == 1 ? t1 : (rsel == 2 ? t2 : t3));
        // bitonic sort, descending, within the 16-lane group
#pragma unroll
        for (int k = 2; k <= 16; k <<= 1)
#pragma unroll
            for (int j = k >> 1; j > 0; j >>= 1) {
                const double o = __shfl_xor(val, j, 64);
                const bool asc = (L16 & k) == 0;
                const bool keep_max = ((L16 & j) == 0) == asc;
                val = keep_max ? fmax(val, o) : fmin(val, o);
            }
        // inclusive prefix sums of the sorted norms
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const double u = __shfl_up(val, o, 16);
            if (L16 >= o) val += u;
        }
        const double v = wave_sum(etr);
        bool ok = v > 0.0;
        #pragma unroll  // constant trip count: the profile stays in registers
        for (int pi = 0; pi < 4; ++pi) {
            if (pi >= pf.np) break;
            const double vr = __shfl(val, pf.rl[pi] - 1, 64);
            ok &= vr > pf.fl[pi] * v * (1.0 + 1e-9);
            kfv[pi] = sqrt(vr);
        }
        fast_reg = ok;
        if (!fast_reg) {  // the eigendecomposition needs all of F
            load_q(1);
            warm_half(1);
            store_f();
        }
        if (lane == 0) flag_fast = fast_reg;
        __syncthreads();
    } else {
        if (warm) store_f();
        if (!INIT && !nuc) {
            if (lane < ZT) {
                double d = 0.0;
                for (int j = 0; j < ZT; ++j) d += cabs2(T0[lane * ZHS + j]);
                wv[lane] = d;
            }
            __syncthreads();
            if (lane < ZT) {
                const double dk = wv[lane];
                int rank = 0;
                for (int j = 0; j < ZT; ++j) rank += (wv[j] > dk) || (wv[j] == dk && j < lane);
                rs2[rank] = dk;
            }
            __syncthreads();
            if (lane == 0) {
                double v = 0.0;
                for (int k = 0; k < ZT; ++k) v += rs2[k];
                int ok = v > 0.0;
                #pragma unroll  // constant trip count: the profile stays in registers
                for (int pi = 0; pi < 4; ++pi) {
                    if (pi >= pf.np) break;
                    double vr = 0.0;
                    for (int k = 0; k < pf.rl[pi]; ++k) vr += rs2[k];
                    ok &= vr > pf.fl[pi] * v * (1.0 + 1e-9);
                }
                flag_fast = ok;
            }
            __syncthreads();
        } else if (lane == 0) {
            flag_fast = 0;
        }
    }
    __syncthreads();
    const bool fast = flag_fast;
#ifdef ACE_DEBUG_SWEEPS
    dbg_fc = __builtin_amdgcn_s_memrealtime();
#endif
    if (lane == 0) flag_any = 0;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    VMax vz, vn;   // max |Z|, |N| of the outputs: the next apply's bound on |Z - N/mu|
    const bool nz_out = pp && fast && flushN;
    if (pp && fast) {   // Z = E: the outputs written in phase 1 stand
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = sacc[q];
        vz = svz;
        if (!flushN) vn = svn;   // else N' is stored as exact zero
    } else {
    if (!fast && !nuc) {
    // H = F F^H (:428), upper blocks (0,0), (0,1), (1,1) -> packed buffer 0
    auto form_h = [&]() {
        d4v hr[3], hi[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int I = q == 2 ? 1 : 0, J = q == 0 ? 0 : 1;
            mm16([&](int r, int k) { return T0[(16 * I + r) * ZHS + k]; },
                 [&](int, int k, int c) { const d2 f = T0[(16 * J + c) * ZHS + k]; return make_double2(f.x, -f.y); },
                 hr[q], hi[q], lane);
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int I = q == 2 ? 1 : 0, J = q == 0 ? 0 : 1;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * I + (lane >> 4) + 4 * r, col = 16 * J + (lane & 15);
                if (row <= col) T0[up_idx(row, col)] = make_double2(hr[q][r], row == col ? 0.0 : hi[q][r]);
            }
        }
        __syncthreads();
    };
    form_h();
    double tr = 0.0;
    if (lane < tx) tr = fabs(T0[up_idx(lane, lane)].x);
    tr = wave_sum(tr);
    const double abs_tol = 1e-18 * tr;
    const int P = tx >> 1;
#ifdef ACE_DEBUG_SWEEPS
    dbg_t1 = __builtin_amdgcn_s_memrealtime();
    sweeps = 0;
#endif
    // rank-one profile ([1] / [0.95]): the top eigenpair by Lanczos (r1_top) instead of every eigenpair
    d2 r1y = make_double2(0.0, 0.0);
    double r1th = 0.0;
    const bool r1 = a.r1lz && pf.np == 1 && pf.rl[0] == 1 && r1_top(T0, T0 + ZPACK, lz_tri, tx, lane, tr, r1y, r1th);
    // the full profile in the cold iterations (ZArgs::tkeig): the top-K eigenpairs by tridiagonal reduction;
    // if its check fails, H is formed again (E from memory, F = Q_prev^H E) for the Jacobi eigensolver
    const int tkK = min(maxr, tx);
    bool tk = false;
    if (!r1 && a.tkeig > 0 && (INIT || a.it <= a.tkeig) && maxr <= TK_MAX && tkK >= 1 && tx >= 2) {
        tk = topk_tri(T0, reinterpret_cast<d2*>(RotS), lz_tri, wv, rs2, scl, tx, tkK, lane, [] { __syncthreads(); });
        if (lane == 0 && a.tkcnt) atomicAdd(a.tkcnt + (tk ? 0 : 1), 1);   // (diagnostics: uses, fallbacks)
        if (!tk) {
            __syncthreads();
            for (int e = lane; e < ZT * ZT; e += 64) {
                const int r = e & 31, c = e >> 5;
                T0[r * ZHS + c] = (r < tx && c < rx) ? evalE(r + tx * c) : zero;
            }
            __syncthreads();
            if (warm) {
                load_q(0);
                load_q(1);
                warm_half(0);
                warm_half(1);
                store_f();
            }
            form_h();
        }
    }
    if (!r1 && !tk) {

    // ---- Jacobi sweeps in the position frame (see ace_zprox.hip for the scheme)
    const int kl = lane & 15, g = lane >> 4;
    // R (position frame), rows i = g + 4r, columns (2kl, 2kl+1)
    double Rt[8][2], Rb[8][2];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int i = g + 4 * r;
        Rt[r][0] = (i == 2 * kl) ? 1.0 : 0.0;
        Rt[r][1] = 0.0;
        Rb[r][0] = (i == 2 * kl + 1) ? 1.0 : 0.0;
        Rb[r][1] = 0.0;
    }
    // this lane's H blocks: off-diagonal slots lane, lane + 64 (a < b); the diagonal block of pair kl
    // (pkd) is updated by the lanes that form that pair's rotation
    int ta[2], tb[2];
    unsigned pk[2][4], pkd[4];   // rd | wr << 11 | (write conj) << 22 | (diag block) << 23
    auto pack = [&](int sa, int sb, unsigned (&o)[4]) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 2 * sa + (r >> 1), j = 2 * sb + (r & 1);
            const unsigned rd = i <= j ? up_idx(i, j) : up_idx(j, i);
            const int ii = circ_next(tx, i), jj = circ_next(tx, j);
            const unsigned wr = ii <= jj ? up_idx(ii, jj) : up_idx(jj, ii);
            o[r] = rd | (wr << 11) | ((ii <= jj ? 0u : 1u) << 22) | ((sa == sb ? 1u : 0u) << 23);
        }
    };
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int e = lane + 64 * q;
        ta[q] = -1;
        tb[q] = 0;
        if (e < 120) {
            const int A_ = c_off_a[e], B_ = c_off_b[e];
            if (B_ < P) {
                ta[q] = A_;
                tb[q] = B_;
            }
        }
        pack(ta[q] < 0 ? 0 : ta[q], ta[q] < 0 ? 1 : tb[q], pk[q]);
    }
    pack(kl < P ? kl : 0, kl < P ? kl : 0, pkd);
    const int rp = up_idx(2 * kl, 2 * kl), rq = up_idx(2 * kl + 1, 2 * kl + 1), rc = up_idx(2 * kl, 2 * kl + 1);
    int cur = 0;
    for (; sweeps < 40; ++sweeps) {
        // convergence pre-check over the off-diagonal entries of this lane's blocks
        bool need = false;
        {
            const d2* H = T0 + cur * ZPACK;
            if (kl < P) need = needs_rot(H[rp].x, H[rq].x, H[rc], abs_tol);   // the pair's own entry
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (ta[q] < 0) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 2 * ta[q] + (r >> 1), j = 2 * tb[q] + (r & 1);
                    if (i < j) need |= needs_rot(H[up_idx(i, i)].x, H[up_idx(j, j)].x, H[up_idx(i, j)], abs_tol);
                }
            }
        }
        if (!__any(need)) break;
        for (int s = 0; s < tx - 1; ++s) {
            const d2* H = T0 + cur * ZPACK;
            d2* Hn = T0 + (cur ^ 1) * ZPACK;
            Rot Jl{1.0, 0.0, make_double2(1.0, 0.0), false};
            const d2 hp = H[rp], hq = H[rq], hc = H[rc];
            if (kl < P) Jl = make_rot(hp.x, hq.x, hc, abs_tol);
            if (lane < 16) RotS[lane] = make_double4(Jl.cs, Jl.sn, Jl.e.x, Jl.e.y);
            // H'[a,b] = Ja^H H[a,b] Jb,  J = [[cs, sn], [-sn e*, cs e*]] (the block update below; the
            // same expressions for the diagonal block of pair kl, Ja = Jb = Jl, written by row 0)
            auto blk = [&](double4 ra, double4 rb, d2 h00, d2 h01, d2 h10, d2 h11, d2& n00, d2& n01, d2& n10,
                           d2& n11) {
                const d2 ebc = make_double2(rb.z, -rb.w), ea = make_double2(ra.z, ra.w);
                const d2 t01 = cmul(h01, ebc), t11 = cmul(h11, ebc);
                const d2 T00 = csub(cscale(h00, rb.x), cscale(t01, rb.y));
                const d2 T01 = cadd(cscale(h00, rb.y), cscale(t01, rb.x));
                const d2 T10 = csub(cscale(h10, rb.x), cscale(t11, rb.y));
                const d2 T11 = cadd(cscale(h10, rb.y), cscale(t11, rb.x));
                const d2 u10 = cmul(ea, T10), u11 = cmul(ea, T11);
                n00 = csub(cscale(T00, ra.x), cscale(u10, ra.y));
                n01 = csub(cscale(T01, ra.x), cscale(u11, ra.y));
                n10 = cadd(cscale(T00, ra.y), cscale(u10, ra.x));
                n11 = cadd(cscale(T01, ra.y), cscale(u11, ra.x));
            };
            auto put = [&](unsigned pw, d2 v) {
                Hn[(pw >> 11) & 2047u] = make_double2(v.x, ((pw >> 22) & 1u) ? -v.y : v.y);
            };
            if (lane < 16 && kl < P) {
                const double4 rl = make_double4(Jl.cs, Jl.sn, Jl.e.x, Jl.e.y);
                d2 n00, n01, n10, n11;
                blk(rl, rl, hp, hc, make_double2(hc.x, -hc.y), hq, n00, n01, n10, n11);
                put(pkd[0], n00);
                put(pkd[1], n01);
                put(pkd[3], n11);
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (ta[q] < 0) continue;
                const double4 ra = RotS[ta[q]], rb = RotS[tb[q]];
                const unsigned p0 = pk[q][0], p1 = pk[q][1], p2 = pk[q][2], p3 = pk[q][3];
                const d2 h00 = H[p0 & 2047u], h01 = H[p1 & 2047u], h11 = H[p3 & 2047u];
                const d2 h10 = H[p2 & 2047u];
                d2 n00, n01, n10, n11;
                blk(ra, rb, h00, h01, h10, h11, n00, n01, n10, n11);
                put(p0, n00);
                put(p1, n01);
                put(p3, n11);
                put(p2, n10);
            }
            // R <- R J for this lane's column pair, then the circle-method column permutation
            {
                const double cs = Jl.cs, sn = Jl.sn, ex = Jl.e.x, ey = -Jl.e.y;  // e* = (ex, ey)
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const double tpr = Rt[r][0], tpi = Rt[r][1];
                    const double bqr = Rb[r][0] * ex - Rb[r][1] * ey, bqi = Rb[r][0] * ey + Rb[r][1] * ex;
                    Rt[r][0] = cs * tpr - sn * bqr;
                    Rt[r][1] = cs * tpi - sn * bqi;
                    Rb[r][0] = sn * tpr + cs * bqr;
                    Rb[r][1] = sn * tpi + cs * bqi;
                }
                // new top(k) = top(0) | bot(0) | top(k-1) for k = 0 | 1 | >=2; new bot(k) = bot(k+1) | top(P-1).
                // The shifts run on every lane (DPP sources must be active); lanes k >= P keep theirs.
                const bool act = P > 1 && kl < P;
                // every lane of each 16-lane row takes part when tx = 32 (P = 16): that case runs
                // without the per-lane masking selects
                auto shift = [&](bool all) {
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    {
                        // one shift for the top row: lane 0 sends its bottom column (new top(1) =
                        // bot(0)), every other lane its top column (new top(k) = top(k-1))
                        const double s0 = kl == 0 ? Rb[r][0] : Rt[r][0], s1 = kl == 0 ? Rb[r][1] : Rt[r][1];
                        const double st0 = dpp_shr1(s0), st1 = dpp_shr1(s1);
                        const double lb0 = dpp_shl1(Rb[r][0]), lb1 = dpp_shl1(Rb[r][1]);
                        const double nt0 = kl == 0 ? Rt[r][0] : st0;
                        const double nt1 = kl == 0 ? Rt[r][1] : st1;
                        const double nb0 = kl == P - 1 ? Rt[r][0] : lb0;
                        const double nb1 = kl == P - 1 ? Rt[r][1] : lb1;
                        if (all || act) {
                            Rt[r][0] = nt0;
                            Rt[r][1] = nt1;
                            Rb[r][0] = nb0;
                            Rb[r][1] = nb1;
                        }
                    }
                }
                };
                if (P == 16) {
                    // tx = 32: the rows' ends are the circle's ends, so the DPP moves' own row-end
                    // behaviour supplies new top(0) = top(0) and new bot(15) = top(15) (the same
                    // permutation as shift(true), without its selects)
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        const double s0 = kl == 0 ? Rb[r][0] : Rt[r][0], s1 = kl == 0 ? Rb[r][1] : Rt[r][1];
                        const double nt0 = dpp_shr1_keep(Rt[r][0], s0), nt1 = dpp_shr1_keep(Rt[r][1], s1);
                        const double nb0 = dpp_shl1_keep(Rt[r][0], Rb[r][0]), nb1 = dpp_shl1_keep(Rt[r][1], Rb[r][1]);
                        Rt[r][0] = nt0;
                        Rt[r][1] = nt1;
                        Rb[r][0] = nb0;
                        Rb[r][1] = nb1;
                    }
                } else {
                    shift(false);
                }
            }
            cur ^= 1;
            __syncthreads();
        }
    }
    if (sweeps >= 40 && lane == 0) atomicOr(&st->status, (int)ACE_ST_EIG_NOCONV);
#ifdef ACE_DEBUG_SWEEPS
    dbg_t2 = __builtin_amdgcn_s_memrealtime();
#endif

    // ---- eigen order (LAPACK ascending, then MATLAB's stable descending sort, :429-430)
    if (lane < tx) wv[lane] = T0[cur * ZPACK + up_idx(lane, lane)].x;
    __syncthreads();
    if (lane < tx) {
        const double wk = wv[lane];
        int asc = 0;
        for (int j = 0; j < tx; ++j) asc += (wv[j] < wk) || (wv[j] == wk && j < lane);
        ascp[lane] = asc;
    }
    __syncthreads();
    if (lane < tx) {
        const double sk = fmax(0.0, wv[lane]);
        const int asc = ascp[lane];
        int rank = 0;
        for (int j = 0; j < tx; ++j) {
            const double sj = fmax(0.0, wv[j]);
            rank += (sj > sk) || (sj == sk && ascp[j] < asc);
        }
        ord[rank] = lane;
    }
    if (lane < ZT) scl[lane] = 1.0;
    __syncthreads();
    if (lane == 0) {  // rank-profile tail rescaling (:469-480), sequential sums
        for (int k = 0; k < tx; ++k) rs2[k] = fmax(0.0, wv[ord[k]]);
        #pragma unroll  // constant trip count: the profile stays in registers
        for (int pi = 0; pi < 4; ++pi) {
            if (pi >= pf.np) break;
            const int r = pf.rl[pi];
            const double f = pf.fl[pi];
            double vr = 0.0, v = 0.0;
            for (int k = 0; k < r; ++k) vr += rs2[k];
            for (int k = 0; k < tx; ++k) v += rs2[k];
            if (vr < v * f) {
                const double sc = fmin(1.0, vr / (v - vr) * (1.0 / f - 1.0));
                for (int k = r; k < tx; ++k) {
                    rs2[k] *= sc;
                    scl[ord[k]] *= sc;
                }
            }
        }
        int any = 0;
        for (int k = 0; k < tx; ++k) any |= scl[k] < 1.0;
        flag_any = any;
    }
    // ---- R -> T0, Qnew = Qprev R -> T0 and global (next iteration's warm start)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int i = g + 4 * r;
        T0[i * ZHS + 2 * kl] = make_double2(Rt[r][0], Rt[r][1]);
        T0[i * ZHS + 2 * kl + 1] = make_double2(Rb[r][0], Rb[r][1]);
    }
    } else if (tk) {
        // the reference's rescale (:469-480) on the top-K eigenvalues (descending, clipped at 0 as :429) and
        // the tail past K as one sum, v = trace(H) - (top-K sum): groups inside the top K get their own
        // factors, the tail (and the completion columns of R) the common one; R's columns are in order
        if (lane == 0) {
            const double* thk = lz_tri + 64;
            double* s2 = wv;   // (topk_tri is done with its LDS arrays)
            double top = 0.0;
            for (int k = 0; k < tkK; ++k) {
                s2[k] = fmax(0.0, thk[k]);
                top += s2[k];
            }
            double tail = fmax(0.0, tr - top), stail = 1.0;
            for (int k = 0; k < ZT; ++k) scl[k] = 1.0;
#pragma unroll  // constant trip count: the profile stays in registers
            for (int pi = 0; pi < 4; ++pi) {
                if (pi >= pf.np) break;
                const int r = pf.rl[pi];
                const double f = pf.fl[pi];
                double vr = 0.0, v = 0.0;
                for (int k = 0; k < tkK; ++k) {
                    if (k < r) vr += s2[k];
                    v += s2[k];
                }
                v += tail;
                if (vr < v * f) {
                    const double sc = fmin(1.0, vr / (v - vr) * (1.0 / f - 1.0));
                    for (int k = r; k < tkK; ++k) {
                        s2[k] *= sc;
                        scl[k] *= sc;
                    }
                    tail *= sc;
                    stail *= sc;
                }
            }
            for (int k = tkK; k < tx; ++k) scl[k] = stail;
            int any = 0;
            for (int k = 0; k < tx; ++k) any |= scl[k] < 1.0;
            flag_any = any;
        }
        if (lane < ZT) ord[lane] = lane;
    } else {
        // the reference's rescale (:469-480) with vr = lambda_1 = theta and v = trace(H) = the eigenvalue sum:
        // every eigenvalue but the largest scaled by c; then Qnew = Qprev Hw with the Householder
        // reflector Hw = I - 2 w w^H / (w^H w), w = y + phi e_1 (phi = y_0 / |y_0|): Hw y = -phi e_1, so
        // column 0 of Qnew is the top eigenvector (up to a phase) and Z = Qnew diag(sqrt(scl)) Qnew^H E
        __syncthreads();
        if (lane == 0) {
            const double f = pf.fl[0], vr = r1th;
            double c = 1.0;
            if (vr < tr * f) c = fmin(1.0, vr / (tr - vr) * (1.0 / f - 1.0));
            flag_any = c < 1.0;
            lz_tri[0] = c;
        }
        d2* wsh = reinterpret_cast<d2*>(RotS);   // 32 complex
        const double y0r = __shfl(r1y.x, 0, 64), y0i = __shfl(r1y.y, 0, 64);
        const double a0 = sqrt(y0r * y0r + y0i * y0i);
        const d2 phi = a0 > 0.0 ? make_double2(y0r / a0, y0i / a0) : make_double2(1.0, 0.0);
        if (lane < 32) wsh[lane] = lane == 0 ? cadd(r1y, phi) : r1y;
        __syncthreads();
        const double c = lz_tri[0];
        if (lane < ZT) {
            scl[lane] = lane == 0 ? 1.0 : c;
            ord[lane] = lane;
        }
        const double f2 = 2.0 / (2.0 + 2.0 * a0);   // 2 / (w^H w), ||y|| = 1
        for (int e = lane; e < ZT * ZT; e += 64) {
            const int i = e >> 5, j = e & 31;
            const d2 wi = wsh[i], wj = wsh[j];
            const d2 p = make_double2(wi.x * wj.x + wi.y * wj.y, wi.y * wj.x - wi.x * wj.y);   // w_i conj(w_j)
            T0[i * ZHS + j] = make_double2((i == j ? 1.0 : 0.0) - f2 * p.x, -f2 * p.y);
        }
    }
    __syncthreads();
    if (warm) {
#pragma unroll
        for (int I = 0; I < 2; ++I)
#pragma unroll
            for (int J = 0; J < 2; ++J)
                mm16([&](int r, int k) { return qprev(16 * I + r, k); },
                     [&](int, int k, int c) { return T0[k * ZHS + 16 * J + c]; }, cr[I][J], ci[I][J], lane);
        __syncthreads();
#pragma unroll
        for (int I = 0; I < 2; ++I)
#pragma unroll
            for (int J = 0; J < 2; ++J)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    T0[(16 * I + (lane >> 4) + 4 * r) * ZHS + 16 * J + (lane & 15)] =
                        make_double2(cr[I][J][r], ci[I][J][r]);
        __syncthreads();
    }
    if (a.Q) {
        // columns in descending eigenvalue order (ord), for the top-16 certificate above
        for (int e = lane; e < tx * tx; e += 64) Qg[e] = T0[(e / tx) * ZHS + ord[e % tx]];
    }
#ifdef ACE_DEBUG_SWEEPS
    dbg_t3 = __builtin_amdgcn_s_memrealtime();
#endif
    }  // !fast
    __syncthreads();

    // per-element update + reductions: nX2, nZ2, nJN2, dZ2.  Whether this iterate becomes
    // opt_X (:344-351) depends only on the Y-step's objective, so it is decided here and X is
    // copied in the same pass that reads it (iter_control below makes the same decision).
    // emit_v: element k with its X, N, Z_old already loaded (opt_X was copied in phase 1)
    auto emit_v = [&](int k, d2 x, d2 nn, d2 zo, d2 znew) {
        if (defer_opt) oX[k] = x;   // Z' != X on this path: the copy cannot be deferred
        vz.add(znew);
        if (!INIT) {
            const d2 d = csub(x, znew);
            const d2 nnew = cadd(nn, cscale(d, mu));
            Nn[k] = nnew;
            vn.add(nnew);
            acc[0] += cabs2(x);
            acc[1] += cabs2(znew);
            acc[2] += cabs2(d);
            acc[3] += cabs2(csub(znew, zo));
        }
        Zn[k] = znew;
    };
    auto emit = [&](int k, d2 znew) {
        const d2 nn = INIT ? zero : N[k], zo = INIT ? zero : Z[k];
        emit_v(k, loadx(k, nn, zo), nn, zo, znew);
    };
    if (flag_any) {
        // per column block J of E: T(:, J) = diag(sqrt(scl)) Qnew^H E(:, J) (rows = eigen indices),
        // then Z^T(J, :) = T(:, J)^T Qnew^T with A = T^T straight from the accumulators and
        // B = Qnew^T from T0.  Output block (J, I): row j (Z column), col i (Z row), so the
        // vec index i + tx*j runs along the lanes.
#pragma unroll
        for (int J = 0; J < 2; ++J) {
#pragma unroll
            for (int K = 0; K < 2; ++K) {
                mm16([&](int r, int k) { const d2 q = T0[k * ZHS + 16 * K + r]; return make_double2(q.x, -q.y); },
                     [&](int, int k, int c) {
                         const int j = 16 * J + c;
                         return (k < tx && j < rx) ? evalE(k + tx * j) : zero;
                     },
                     cr[K][0], ci[K][0], lane);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double w = sqrt(scl[16 * K + (lane >> 4) + 4 * r]);
                    cr[K][0][r] *= w;
                    ci[K][0][r] *= w;
                }
            }
#pragma unroll
            for (int I = 0; I < 2; ++I) {
                d4v zr = {0.0, 0.0, 0.0, 0.0}, zi = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int K = 0; K < 2; ++K)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int kk = 16 * K + 4 * q + (lane >> 4);
                        const d2 av = make_double2(cr[K][0][q], ci[K][0][q]);       // T[kk][16J + (lane&15)]
                        const d2 bv = T0[(16 * I + (lane & 15)) * ZHS + kk];          // Qnew[16I + c][kk]
                        mfma_c(av, bv, zr, zi);
                    }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = 16 * J + (lane >> 4) + 4 * r, i = 16 * I + (lane & 15);
                    if (i < tx && j < rx) emit(i + tx * j, make_double2(zr[r], zi[r]));
                }
            }
        }
    } else {
        // Z = E: all loads of a chunk are issued before any of its stores (the stores to N, Z and
        // opt_X would otherwise serialise every element behind a full memory round trip)
        // (nuclear r = 1: Z = E f with f = max(0, ||E|| - 1/mu) / ||E||, the SVD soft threshold of
        // the n x 1 iterate, inferLowRank_Nuclear.m:415-417)
        double fz = 1.0;
        if (nuc) {
            const double nzv = sqrt(wave_sum(etr));
            fz = nzv > 0.0 ? fmax(0.0, nzv - imu) / nzv : 0.0;
        }
        constexpr int CH = 8;
        for (int k0 = 0; k0 < n; k0 += 64 * CH) {
            d2 xv[CH], nv[CH], zv[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int k = k0 + lane + 64 * u;
                xv[u] = nv[u] = zv[u] = zero;
                if (k < n) {
                    xv[u] = X[k];
                    nv[u] = N[k];
                    if (!INIT) zv[u] = Z[k];
                }
            }
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int k = k0 + lane + 64 * u;
                const d2 x = wm ? xw(zv[u], nv[u], xv[u], imu) : xv[u];
                const d2 e = make_double2(fma(nv[u].x, imu, x.x), fma(nv[u].y, imu, x.y));
                if (k < n) emit_v(k, x, nv[u], zv[u], nuc ? cscale(e, fz) : e);
            }
        }
    }
    }  // !(fast)
#ifdef ACE_DEBUG_SWEEPS
    const unsigned long long dbg_t4 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && (b == 0 || b == 2000) && (a.it < 30 || a.it % 20 == 0))
        printf("1w b %d it %d sweeps %d pre %llu jac %llu order+Q %llu emit %llu (x10ns) scaled %d\n", b, a.it, sweeps,
               dbg_t1 - dbg_t0, dbg_t2 - dbg_t1, dbg_t3 - dbg_t2, dbg_t4 - dbg_t3, flag_any);
    if (lane == 0 && a.it >= 1 && a.it <= 8 && (b & 127) == 5) printf("cold b %d it %d sweeps %d scaled %d\n", b, a.it, sweeps, flag_any);
    if (lane == 0 && (b == 0 || b == 2000) && (a.it % 20 == 0))
        printf("1w b %d it %d fast: E %llu F %llu cert %llu rest %llu\n", b, a.it, dbg_fa - dbg_t0, dbg_fb - dbg_fa,
               dbg_fc - dbg_fb, dbg_t4 - dbg_fc);
#endif
    // bound for the next iteration's V = Z - N/mu (after iter_control's mu update).  A convergence
    // test left pending (RealState::dpend) may still multiply mu by rho in the next gyk_kernel
    // (dual_finish): the bound takes the smaller of the two mu values (the same mu for rho >= 1)
    auto write_vbound = [&]() {
        const double zm = wave_max(vz.m), nm = wave_max(vn.m), sn = wave_sum(vz.s + vn.s);
        if (lane == 0) {
            const double mu_lo = st->dpend ? fmin(st->mu, st->mu * a.rho) : st->mu;
            st->vbound = (zm + nm * (1.0 / mu_lo)) * (1.0 + 0x1p-40) + sn;
        }
    };
    if (INIT) {
        write_vbound();   // N = 0 after init (init_r_kernel)
        return;
    }

    const double s_nX2 = wave_sum(acc[0]), s_nZ2 = wave_sum(acc[1]), s_jn2 = wave_sum(acc[2]),
                 s_dZ2 = wave_sum(acc[3]), s_dAtY = wave_sum(dAtY), s_nAtY = wave_sum(nAtY);
    int improved = 0;
    if (lane == 0)
        improved = iter_control(a, st, mu, s_nX2, s_nZ2, s_jn2, s_dZ2, s_dAtY, s_nAtY);
    improved = __shfl(improved, 0, 64);
    if ((improved & 2) && a.fixup_now) dual_fixup(a, b, st);   // pending test at the last iteration
    write_vbound();
    if (lane == 0) {
        st->nzero = nz_out ? 1 : 0;
        st->avok = (nz_in && nz_out) ? 1 : 0;   // V' = Z' = E = X: A V' is the Y-step's AX
        // the next iteration's E starts from Z' = E of this one: a fresh perturbation reference
        const bool kok = nz_out && top16 && fast_reg;
        st->kfok = kok ? 1 : 0;
        st->kfcum = 0.0;
#pragma unroll
        for (int pi = 0; pi < 4; ++pi) st->kf[pi] = kok ? kfv[pi] : 0.0;
        if (improved_pre) optsrc = (defer_opt && pp && fast) ? zn_id : 0;
        st->optsrc = optsrc;
    }
#ifdef ACE_DEBUG_SWEEPS
    if (lane == 0 && a.it == 100) {
        const unsigned long long te = __builtin_amdgcn_s_memrealtime();
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        printf("wave %d %llu %llu %u\n", b, dbg_t0, te, hw);
    }
#endif
}

template <bool INIT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void zstep1w_kernel(ZArgs a) {
    zstep1w_body<INIT>(a, blockIdx.x);
}

// Steady-state form (ZArgs::compact): one wave per ZC realisations.  Lane i settles realisation
// b0 + i when the lean kernel or the fused apply_AH left it certifiable (the control runs on the
// lanes in parallel); the wave then runs the full one-wave Z-step for the others, one after
// another.  A launch of nb / ZC waves instead of nb: in the steady state every realisation is
// settled on its lane, and a fallback (rare after the cold start) costs a sequential step.
constexpr int ZC = 8;
__device__ __noinline__ void zstep1w_body_call(const ZArgs& a, int b) { zstep1w_body<false>(a, b); }
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void zstep1w_compact_kernel(ZArgs a, int nb) {
    const int lane = threadIdx.x, b0 = blockIdx.x * ZC;
    int full = 0;
    if (lane < ZC && b0 + lane < nb) {
        const int b = b0 + lane;
        RealState* st = a.st + b;
        if (!st->done && !(a.lean && st->zit >= a.it)) {
            full = 1;
            if (a.xfuse && st->fzit == a.it) full = !fused_control(a, st, z_profile(a, b));
        }
    }
    unsigned long long m = __ballot(full);
    while (m) {
        const int i = __ffsll((long long)m) - 1;
        m &= m - 1;
        zstep1w_body_call(a, b0 + i);   // (re-checks the fused bound: it fails again, X from Z')
        __syncthreads();
    }
}

// ---- lean steady-state Z-step (A2only, wmode, ping-pong, N = 0 on entry).
// In the steady state of the unit solve N = 0, so E = X = Z + W and the reference's Z-prox
// leaves Z = E unless its tail rescaling fires (:469-484).  The full kernel above proves that
// it does not with the Ky Fan certificate on F = Qprev^H E (Q loads, MFMA, sort).  Here the
// proof is a perturbation bound instead: with S_p the r_p rows that certified E_ref,
//   sqrt(sum of the r_p largest eigenvalues of E E^H) >= ||P_S Qprev^H E|| >= kf[p] - ||E - E_ref||
//                                                       >= kf[p] - sum_i ||E_i - E_{i-1}||
// and ||E_i - E_{i-1}|| = ||X - Z|| is the Z-step's own dZ2 term, so a certified realisation
// costs one pass over W and Z (read) and Z' (write).  kf is 1e-12 relatively deflated and the
// certificate keeps the full kernel's 1e-9 margin.  The element order and sums are those of
// the full kernel's phase 1 (e = lane + 64 t), so for tx = 32 its outputs are bit-identical
// to the full kernel's; a realisation the bound cannot certify writes nothing but the
// speculative Z' (which the full kernel rewrites) and is left to zstep1w_kernel.
constexpr int ZL_WAVES = 4;
#ifdef ACE_LEAN_STAMPS
#define LSTAMP(i) do { ts_[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define LSTAMP(i)
#endif
__global__ __launch_bounds__(64 * ZL_WAVES) __attribute__((amdgpu_waves_per_eu(2))) void zlean_kernel(ZArgs a, int nb) {
    const int lane = threadIdx.x & 63, b = min(blockIdx.x * ZL_WAVES + (int)(threadIdx.x >> 6), nb - 1);
    if (blockIdx.x * ZL_WAVES + (int)(threadIdx.x >> 6) >= nb) return;
#ifdef ACE_LEAN_STAMPS
    unsigned long long ts_[5] = {};
#endif
    LSTAMP(0);
    const int n = a.n;
    // W and Z of the whole realisation (n = tx rx <= 1024, e = lane + 64 u) are requested with
    // its state, so the wave's latency is about one round trip; an ineligible realisation drops
    // its loads.
    RealState* st = a.st + b;
    const int done = st->done, kfok = st->kfok, nzero = st->nzero, optsrc0 = st->optsrc;
    const double mu = st->mu, kfcum = st->kfcum, dAtY = st->dAtY, nAtY = st->nAtY;
    const double kf0 = st->kf[0], kf1 = st->kf[1], kf2 = st->kf[2], kf3 = st->kf[3];
    const IterIn itin = iter_in(st);
    const double obj2 = itin.obj2, opt_obj = itin.opt_obj;
    const ZProfile pf = z_profile(a, b);
    constexpr int LE = 16;
    const d2* W = reinterpret_cast<const d2*>(a.X) + (long long)b * n;
    const d2* Z = reinterpret_cast<const d2*>(a.Z) + (long long)b * n;
    d2 wv[LE], zv[LE];
    const int le = n >> 6;   // launch_zlean: n is a multiple of 64
#pragma unroll
    for (int u = 0; u < LE; ++u) {
        wv[u] = zv[u] = make_double2(0.0, 0.0);
        if (u < le) {
            wv[u] = W[lane + 64 * u];
            zv[u] = Z[lane + 64 * u];
        }
    }
    const int zn_id = 1 + (a.it & 1);
    if (done || !kfok || !nzero) return;
    LSTAMP(1);
    const double imu = 1.0 / mu;
    d2* Zn = reinterpret_cast<d2*>(a.Zn) + (long long)b * n;
    d2* oX = reinterpret_cast<d2*>(a.optX) + (long long)b * n;
    d2* Xc = reinterpret_cast<d2*>(a.Xcur) + (long long)b * n;
    int optsrc = optsrc0;
    if (optsrc == zn_id) {   // the Z' buffer holds the best iterate: keep it before overwriting
        for (int k = lane; k < n; k += 64 * 4) {
            const d2 v0 = Zn[k], v1 = Zn[min(k + 64, n - 1)], v2 = Zn[min(k + 128, n - 1)],
                     v3 = Zn[min(k + 192, n - 1)];
            oX[k] = v0;
            if (k + 64 < n) oX[k + 64] = v1;
            if (k + 128 < n) oX[k + 128] = v2;
            if (k + 192 < n) oX[k + 192] = v3;
        }
        optsrc = 0;
        if (lane == 0) st->optsrc = 0;   // now, for the full kernel if the bound fails below
    }
    const bool improved_pre = sqrt(obj2) < opt_obj;
    const bool keep_cur = !improved_pre && !(opt_obj < INFINITY);   // finalize's fallback X
    const d2 zero = make_double2(0.0, 0.0);
    double sacc[4] = {0.0, 0.0, 0.0, 0.0}, etr = 0.0;
    VMax svz;
#pragma unroll
    for (int u = 0; u < LE; ++u) {
        const int k = lane + 64 * u;
        if (u >= le) continue;
        const d2 x = xw(zv[u], zero, wv[u], imu);
        const d2 ev = make_double2(fma(0.0, imu, x.x), fma(0.0, imu, x.y));   // E = X + N/mu, N = 0
        etr += cabs2(ev);
        if (keep_cur) Xc[k] = x;
        Zn[k] = ev;
        const d2 d = csub(x, ev);
        sacc[0] += cabs2(x);
        sacc[1] += cabs2(ev);
        sacc[2] += cabs2(d);
        sacc[3] += cabs2(csub(ev, zv[u]));
        svz.add(ev);
    }
    const double v = wave_sum(etr), s_nX2 = wave_sum(sacc[0]), s_nZ2 = wave_sum(sacc[1]),
                 s_jn2 = wave_sum(sacc[2]), s_dZ2 = wave_sum(sacc[3]);
    LSTAMP(2);
    const double cum = (kfcum + sqrt(s_dZ2)) * (1.0 + 0x1p-40);
    bool ok = v > 0.0;
#pragma unroll
    for (int pi = 0; pi < 4; ++pi) {
        if (pi >= pf.np) break;
        const double kfp = pi == 0 ? kf0 : (pi == 1 ? kf1 : (pi == 2 ? kf2 : kf3));
        const double lb = kfp * (1.0 - 1e-12) - cum;
        ok &= lb > 0.0 && lb * lb > pf.fl[pi] * v * (1.0 + 1e-9);
    }
    if (!ok) return;   // zstep1w_kernel redoes this realisation (Z' is rewritten there)
    const double zm = wave_max(svz.m), sn = wave_sum(svz.s);
    LSTAMP(3);
    int ctl = 0;
    if (lane == 0) {
        ctl = iter_control_in(a, st, itin, mu, s_nX2, s_nZ2, s_jn2, s_dZ2, dAtY, nAtY);
        st->vbound = zm * (1.0 + 0x1p-40) + sn;   // N' = 0: the bound on V' = Z' - N'/mu' is max|Z'|
        st->nzero = 1;
        st->avok = 1;
        if (improved_pre) optsrc = zn_id;   // deferred opt_X: X = Z' bit for bit
        st->optsrc = optsrc;
        st->kfcum = cum;
        st->zit = a.it;
    }
    if ((__shfl(ctl, 0, 64) & 2) && a.fixup_now) dual_fixup(a, b, st);   // pending test at the last iteration
    LSTAMP(4);
#ifdef ACE_LEAN_STAMPS
    if (lane == 0 && a.it == 100 && (b % 97) == 3) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        printf("lean b %d t0 %llu ld %llu sum %llu chk %llu ctl %llu hw %x\n", b, ts_[0], ts_[1] - ts_[0], ts_[2] - ts_[1],
               ts_[3] - ts_[2], ts_[4] - ts_[3], hw);
    }
#endif
}

}  // namespace

void launch_zlean(const ZArgs& a, int batch, hipStream_t st) {
    if (a.n % 64 != 0 || a.n > 1024) return;   // the full kernel handles every realisation
    hipLaunchKernelGGL(zlean_kernel, dim3((batch + ZL_WAVES - 1) / ZL_WAVES), dim3(64 * ZL_WAVES), 0, st, a, batch);
}

void launch_zstep1w(bool init, const ZArgs& a, int batch, hipStream_t st) {
    if (init) hipLaunchKernelGGL(zstep1w_kernel<true>, dim3(batch), dim3(64), 0, st, a);
    else if (a.compact) hipLaunchKernelGGL(zstep1w_compact_kernel, dim3((batch + ZC - 1) / ZC), dim3(64), 0, st, a, batch);
    else hipLaunchKernelGGL(zstep1w_kernel<false>, dim3(batch), dim3(64), 0, st, a);
}

}  // namespace ace
