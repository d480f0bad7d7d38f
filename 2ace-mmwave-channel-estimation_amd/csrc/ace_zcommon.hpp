// Helpers shared by the Z-prox kernels (ace_zprox.hip, ace_zprox1w.hip): Jacobi
// rotations, packed-triangular indexing, the circle-method position map.
#pragma once
#include "ace_common.hpp"

namespace ace {
namespace {


constexpr int ZT = 32;            // padded tile size (tx, rx <= 32)
constexpr int ZHS = ZT + 1;       // LDS row stride (complex) of a 32x32 tile
constexpr int ZPACK = 528;        // packed upper triangle of a 32x32 matrix

// upper-triangular enumeration of the 16x16 slot-pair blocks (ka <= kb)
static __constant__ unsigned char c_tri_a[136] = {0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,2,2,2,2,2,2,2,2,2,2,2,2,2,2,3,3,3,3,3,3,3,3,3,3,3,3,3,4,4,4,4,4,4,4,4,4,4,4,4,5,5,5,5,5,5,5,5,5,5,5,6,6,6,6,6,6,6,6,6,6,7,7,7,7,7,7,7,7,7,8,8,8,8,8,8,8,8,9,9,9,9,9,9,9,10,10,10,10,10,10,11,11,11,11,11,12,12,12,12,13,13,13,14,14,15};
static __constant__ unsigned char c_tri_b[136] = {0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,2,3,4,5,6,7,8,9,10,11,12,13,14,15,3,4,5,6,7,8,9,10,11,12,13,14,15,4,5,6,7,8,9,10,11,12,13,14,15,5,6,7,8,9,10,11,12,13,14,15,6,7,8,9,10,11,12,13,14,15,7,8,9,10,11,12,13,14,15,8,9,10,11,12,13,14,15,9,10,11,12,13,14,15,10,11,12,13,14,15,11,12,13,14,15,12,13,14,15,13,14,15,14,15,15};

// Jacobi rotation J = [[cs, sn], [-sn e*, cs e*]] annihilating h_pq of the Hermitian
// 2x2 block [[ap, c], [c*, aq]] (c = |c| e): tan(theta) = t with
// t = sign(aq - ap) 2|c| / (|aq - ap| + sqrt((aq - ap)^2 + 4|c|^2)).
struct Rot {
    double cs, sn;
    d2 e;
    bool on;
};
// v_rsq_f64 / v_rcp_f64 seeds refined by two Newton steps (~1 ulp); operands are
// positive and finite here (guarded by the rotation threshold).
__device__ __forceinline__ double frsq(double x) {
    double y = __builtin_amdgcn_rsq(x);
    y = fma(y * fma(-x * y, y, 1.0), 0.5, y);
    y = fma(y * fma(-x * y, y, 1.0), 0.5, y);
    return y;
}
__device__ __forceinline__ double frcp(double x) {
    double y = __builtin_amdgcn_rcp(x);
    y = fma(y, fma(-x, y, 1.0), y);
    y = fma(y, fma(-x, y, 1.0), y);
    return y;
}
// rotate pair (p,q) unless |h_pq| is negligible: |h_pq| <= 1e-18 tr(H) (absolute, below
// LAPACK's normwise eps) or |h_pq|^2 <= 1e-32 |h_pp h_qq| (relative, the classical
// Jacobi test)
__device__ __forceinline__ bool needs_rot(double ap, double aq, d2 c, double abs_tol) {
    const double ac2 = cabs2(c);
    return ac2 > abs_tol * abs_tol && ac2 > 1e-32 * fabs(ap * aq) && ac2 > 1e-300;
}
__device__ __forceinline__ Rot make_rot(double ap, double aq, d2 c, double abs_tol) {
    Rot r{1.0, 0.0, make_double2(1.0, 0.0), false};
    const double ac2 = cabs2(c);
    if (needs_rot(ap, aq, c, abs_tol)) {
        const double ir = frsq(ac2), ac = ac2 * ir;
        r.e = make_double2(c.x * ir, c.y * ir);
        const double d = aq - ap;
        const double q = fma(d, d, 4.0 * ac2);
        const double D = q * frsq(q);
        double tt = 2.0 * ac * frcp(fabs(d) + D);
        if (d < 0.0) tt = -tt;
        r.cs = frsq(fma(tt, tt, 1.0));
        r.sn = tt * r.cs;
        r.on = true;
    }
    return r;
}

// Packed upper-triangular index of (i, j), i <= j < 32 (528 entries).
__device__ __forceinline__ int up_idx(int i, int j) { return i * 32 - ((i * (i - 1)) >> 1) + (j - i); }

// Circle-method position map for n (even) positions with pairs (2k, 2k+1): position
// 0 is fixed, the "top" elements 2k move right, the "bottom" elements 2k+1 move left.
__device__ __forceinline__ int circ_next(int n, int p) {
    if (n == 2) return p;
    const int P = n >> 1;
    if (p == 0) return 0;
    if (p == 1) return 2;
    if ((p & 1) == 0) return (p == 2 * P - 2) ? 2 * P - 1 : p + 2;
    return p - 2;
}

// Per-iteration control of one realisation, executed by a single thread after the
// Z-step reductions: best-objective bookkeeping (inferLowRankV4_multi.m:344-351),
// residuals (:364-366), thresholds (:368-370), stop test (:372), mu update (:379-381).
// Sums: nX2 = ||X||^2, nZ2 = ||Z||^2, jn2 = ||X - Z||^2, dZ2 = ||Z - Z0||^2,
// dAtY = ||A^H (Y - Y0)||^2, nAtY = ||A^H Y||^2.  Returns bit 0: the objective improved, bit 1:
// the convergence test is pending (ZArgs::lazy_dual; the caller runs dual_fixup on the wave).
// Sum the fused Y-step partials of realisation b (fixed tile order) into v[5].
__device__ __forceinline__ void ystep_sums(const ZArgs& a, int b, double* v) {
    for (int k = 0; k < 5; ++k) v[k] = 0.0;
    for (int t = 0; t < a.ytiles; ++t)
        for (int k = 0; k < 5; ++k) v[k] += a.ypart[((long long)b * a.ytiles + t) * 5 + k];
}

// The inputs iter_control reads from RealState, loaded as one batch (the lean Z-step reads them
// with its other loads: a load issued after the kernel's stores would wait for them to retire).
struct IterIn {
    double obj2, nAX2, nY2, nJM2, dY2, opt_obj, last_res;
    int32_t status;
};
__device__ __forceinline__ IterIn iter_in(const RealState* st) {
    return IterIn{st->obj2, st->nAX2, st->nY2, st->nJM2, st->dY2, st->opt_obj, st->last_res, st->status};
}
// (it: the iteration being controlled, a.it except in msr_kernel, which runs several per launch)
__device__ __forceinline__ int iter_control_in(const ZArgs& a, RealState* st, const IterIn& in, double mu, double nX2,
                                               double nZ2, double jn2, double dZ2, double dAtY, double nAtY, int it) {
    const int m = a.mthr ? a.mthr : a.m, n = a.n;
    const double nX = sqrt(nX2), nZ = sqrt(nZ2);
    const double dAtY2 = fmax(0.0, dAtY), nAtY2 = fmax(0.0, nAtY);
    const double obj = sqrt(in.obj2);
    const double nAX = sqrt(in.nAX2), nY = sqrt(in.nY2);
    const double r = (double)a.r;  // columns per realisation
    int improved = 0;
    if (obj < in.opt_obj) {
        st->opt_obj = obj;
        improved = 1;
    }
    const double res_prim = sqrt(in.nJM2 + jn2);
    const double res_comb = sqrt(res_prim * res_prim + in.dY2 + dZ2);
    if (a.lazy_dual) {
        // (P && D) || C: D is needed only when P holds and C does not (dual_fixup finishes then)
        const double mx1 = fmax(nAX, nY), mx2 = fmax(nX, nZ);
        const double t_prim = a.tol_abs * sqrt((double)(m + n) * r) + a.tol_rel * sqrt(mx1 * mx1 + mx2 * mx2);
        const double t_comb =
            a.tol_abs * sqrt((double)(m + n) * r * 2) + a.tol_rel * sqrt(mx1 * mx1 + mx2 * mx2 + nY * nY + nZ * nZ);
        st->iters = it;
        if (res_prim < t_prim && !(res_comb < t_comb)) {
            st->dpend = 1;
            st->pd_dZ2 = dZ2;
            st->pd_nZ2 = nZ * nZ;
            st->pd_rc = res_comb;
            return improved | 2;   // bit 1: the test is pending (dual_fixup)
        }
        const bool conv = res_comb < t_comb;
        bool stop = false;
        if (conv) {
            st->status = in.status | ACE_ST_CONVERGED;
            if (!a.fixed_iters) stop = true;
        }
        if (stop) {
            st->done = 1;
            atomicAdd(a.done_count, 1);
        } else {
            if (res_comb > in.last_res * 0.9) st->mu = mu * a.rho;
            st->last_res = res_comb;
        }
        return improved;
    }
    const double res_dual = mu * sqrt(dAtY2 + dZ2);
    const double mx1 = fmax(nAX, nY), mx2 = fmax(nX, nZ);
    const double t_prim = a.tol_abs * sqrt((double)(m + n) * r) + a.tol_rel * sqrt(mx1 * mx1 + mx2 * mx2);
    const double t_dual = a.tol_abs * sqrt((double)n * r * 2) + a.tol_rel * sqrt(nAtY2 + nZ * nZ);
    const double t_comb =
        a.tol_abs * sqrt((double)(m + n) * r * 2) + a.tol_rel * sqrt(mx1 * mx1 + mx2 * mx2 + nY * nY + nZ * nZ);
    st->iters = it;
    const bool conv = (res_prim < t_prim && res_dual < t_dual) || (res_comb < t_comb);
    bool stop = false;
    if (conv) {
        st->status = in.status | ACE_ST_CONVERGED;
        if (!a.fixed_iters) stop = true;
    }
    if (stop) {
        st->done = 1;
        atomicAdd(a.done_count, 1);
    } else {
        if (res_comb > in.last_res * 0.9) st->mu = mu * a.rho;
        st->last_res = res_comb;
    }
    return improved;
}
__device__ __forceinline__ int iter_control_in(const ZArgs& a, RealState* st, const IterIn& in, double mu, double nX2,
                                               double nZ2, double jn2, double dZ2, double dAtY, double nAtY) {
    return iter_control_in(a, st, in, mu, nX2, nZ2, jn2, dZ2, dAtY, nAtY, a.it);
}
// Finish a pending convergence test (RealState::dpend) on one wave, for the last iteration
// (ZArgs::fixup_now; before it, gyk_kernel of the next iteration finishes it on the int8
// matrix cores): ||A^H (Y - Y0)||^2 = dY^H K dY and ||A^H Y||^2 = Y^H K Y from the f64 K (rows
// of K^H = K read coalesced), then dual_finish.
__device__ __forceinline__ void dual_fixup(const ZArgs& a, int b, RealState* st) {
    const int lane = threadIdx.x & 63, m = a.m;
    const d2* Yn = reinterpret_cast<const d2*>(a.Ynew) + (long long)b * m;
    const d2* Yo = reinterpret_cast<const d2*>(a.Yold) + (long long)b * m;
    const d2* K = reinterpret_cast<const d2*>(a.Kf);
    double dacc = 0.0, nacc = 0.0;
    for (int i0 = 0; i0 < m; i0 += 64) {
        const int i = i0 + lane, ic = min(i, m - 1);
        double kyr = 0.0, kyi = 0.0, kdr = 0.0, kdi = 0.0;
        for (int k = 0; k < m; ++k) {
            const d2 y = Yn[k], yo = Yo[k], kk = K[(long long)k * m + ic];   // K[ic][k] = conj(kk)
            const double dyr = y.x - yo.x, dyi = y.y - yo.y;
            kyr += kk.x * y.x + kk.y * y.y;
            kyi += kk.x * y.y - kk.y * y.x;
            kdr += kk.x * dyr + kk.y * dyi;
            kdi += kk.x * dyi - kk.y * dyr;
        }
        if (i < m) {
            const d2 y = Yn[i], yo = Yo[i];
            const double dyr = y.x - yo.x, dyi = y.y - yo.y;
            nacc += y.x * kyr + y.y * kyi;
            dacc += dyr * kdr + dyi * kdi;
        }
    }
    const double dAtY = wave_sum(dacc), nAtY = wave_sum(nacc);
    if (lane == 0) dual_finish(DualCtl{a.tol_abs, a.tol_rel, a.rho, a.fixed_iters, a.n, a.r, a.done_count}, st, dAtY, nAtY);
}

__device__ __forceinline__ int iter_control(const ZArgs& a, RealState* st, double mu, double nX2, double nZ2,
                                            double jn2, double dZ2, double dAtY, double nAtY) {
    if (a.ypart) {
        double v[5];
        ystep_sums(a, (int)(st - a.st), v);
        st->obj2 = v[0];
        st->nAX2 = v[1];
        st->nY2 = v[2];
        st->nJM2 = v[3];
        st->dY2 = v[4];
    }
    return iter_control_in(a, st, iter_in(st), mu, nX2, nZ2, jn2, dZ2, dAtY, nAtY);
}

// Certificate and iteration control of a realisation whose X the fused apply_AH formed in Z'
// with its sums (RealState::fzit, fs0 = ||X||^2, fs3 = ||X - Z||^2), or whose sums gyk_kernel
// formed in m-space (RealState::mzit == it, X implicit), on one lane: the perturbation bound of
// zlean_kernel; if it holds, Z' = E = X stands, N' = 0, and the control runs.  Returns 0 (nothing
// written) when the bound fails: the full Z-step must run; else 1, plus 2 when the convergence
// test is left pending (ZArgs::lazy_dual: at the last iteration the wave runs dual_fixup).
// COPY: the state is copied to registers in one batch of loads and written back (the one-wave
// Z-step, scalar loads); otherwise the fields are used in place (gyf_kernel's m-space steps).
template <bool COPY = true>
__device__ __forceinline__ int fused_control(const ZArgs& a, RealState* st, const ZProfile& pf, int it) {
    RealState sc;
    if constexpr (COPY) sc = *st;
    RealState& s = COPY ? sc : *st;
    const double s0 = s.fs0, s3 = s.fs3;
    const double cum = (s.kfcum + sqrt(s3)) * (1.0 + 0x1p-40);
    bool pass = s0 > 0.0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        if (p >= pf.np) break;
        const double lb = s.kf[p] * (1.0 - 1e-12) - cum;
        pass &= lb > 0.0 && lb * lb > pf.fl[p] * s0 * (1.0 + 1e-9);
    }
    pass &= !(a.msp && s.mzit == it && it == a.msp_fail_it);   // (tests: the fallback path)
    if (!pass) return 0;
    const bool improved_pre = sqrt(s.obj2) < s.opt_obj;
    const int optsrc = s.optsrc;   // (the fused kernel kept a best iterate in Z')
    const int ctl = iter_control_in(a, &s, iter_in(&s), s.mu, s0, s0, 0.0, s3, s.dAtY, s.nAtY, it);
    s.vbound = sqrt(s0) * (1.0 + 0x1p-40);   // N' = 0: max|Z'| <= ||Z'|| (NaN-sticky)
    s.nzero = 1;
    s.avok = 1;
    // deferred opt_X: X = Z' bit for bit, or (m-space) X = Z0 + A^H S' with S' in Sg[it & 1]
    s.optsrc = improved_pre ? (a.msp && s.mzit == it ? 4 + (it & 1) : 1 + (it & 1)) : optsrc;
    s.kfcum = cum;
    s.zit = it;
    if constexpr (COPY) *st = sc;
    return 1 | (ctl & 2);
}
template <bool COPY = true>
__device__ __forceinline__ int fused_control(const ZArgs& a, RealState* st, const ZProfile& pf) {
    return fused_control<COPY>(a, st, pf, a.it);
}

}  // namespace
}  // namespace ace
