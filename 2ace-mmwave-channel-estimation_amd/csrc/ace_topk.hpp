// The top-K eigenpairs of a 32 x 32 Hermitian matrix through a one-wave tridiagonal reduction (topk_tri):
// the eigen part of ArgMinZ's full rank profile, shared by the one-wave Z-step (ace_zprox1w.hip) and the
// four-wave r-column Z-step (ace_zprox.hip).
#pragma once
#include "ace_common.hpp"
#include "ace_zcommon.hpp"

namespace ace {
namespace {

__device__ __forceinline__ d2 conj_d2(d2 v) { return make_double2(v.x, -v.y); }

// ---- the full rank profile: the top-K eigenpairs through a tridiagonal reduction ---------------------
// The tail rescaling (:469-480) scales the sorted eigenvalues by one factor per profile group (1..r_0,
// r_0+1..r_1, ...) and every eigenvalue past the largest rank K by one common factor, so Z = U diag(sqrt(
// scale)) U^H E (:482-484) needs the top-K eigenvectors and ANY orthonormal completion of them.  topk_tri
// reduces H to a real tridiagonal T = Q_h^H H Q_h with LAPACK zhetd2's reflectors (lower form; H held in
// registers, lane (i, h) row i, columns 16h..16h+15), finds T's K largest eigenvalues by multisection on
// Sturm counts (two probes per lane), their vectors by twisted factorisation (dlar1v), orthonormalises them
// with a Householder QR whose Q_s also supplies the completion, checks every Ritz residual
// ||T q_j - theta_j q_j|| <= 2^-44 ||T||, and writes R = Q_h Q_s (columns in descending eigenvalue order)
// into T0 as a 32 x ZHS tile, theta_j into tk[64 + j].  A failed check (eigenvalues clustered inside the top
// K, where separate twisted vectors lose orthogonality) returns false with H destroyed: the caller rebuilds
// it and runs the Jacobi eigensolver.  One wave; `sync` orders the wave's LDS traffic.
// LDS: T0 (the packed H on entry, both packed buffers as scratch), vsh (32 complex), tk (>= 64 + TK_MAX
// doubles), dd, ee, e2 (32 doubles each).
constexpr int TK_MAX = 16;   // largest profile rank taken this way (32-antenna profile: K = 12)
constexpr int TK_LD = 65;    // LDS stride (doubles) of the per-eigenvalue vectors (spreads the banks)
constexpr int TK_ONE = 512, TK_ZERO = 513;   // constant slots after the compact reflectors (<= 465 entries)
// sum over each 32-lane half: DPP within the 16-lane rows, then one swizzle across the two rows
__device__ __forceinline__ double hsum32(double v) {   // (the row pair on a permlane16 swap: VALU, no LDS)
    return xor16_sum(bsum16(v));
}
// lane src's value in every lane (src uniform: v_readlane, no LDS round trip)
__device__ __forceinline__ double readlane_d(double x, int src) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), src),
                            __builtin_amdgcn_readlane(__double2loint(x), src));
}
template <class Sync>
__device__ __forceinline__ bool topk_tri(d2* T0, d2* vsh, double* tk, double* dd, double* ee, double* e2, int n, int K,
                                         int lane, Sync sync) {
    const int i = lane & 31, h = lane >> 5, c0 = 16 * h;
    const d2 zero = make_double2(0.0, 0.0), one = make_double2(1.0, 0.0);
#ifdef ACE_DEBUG_TK   // phase times of realisations 5 and 1500 (10 ns units)
    unsigned long long tkt[8];
    int tkn = 0;
    tkt[tkn++] = __builtin_amdgcn_s_memrealtime();
#define TK_STAMP() do { tkt[tkn++] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define TK_STAMP() do { } while (0)
#endif
    d2* VB = T0;   // reflector k: v[k+2..n) at VB[off_k ..] (v[k+1] = 1), off_k = k (n - 2) - k (k - 1) / 2
    double* S = reinterpret_cast<double*>(T0 + ZPACK);   // twisted vectors, TK_LD doubles each
    d2* rowb = T0 + 992;   // (tridiagonalisation only: row k of the reduced matrix, then w)
    d2* wsh = T0 + 1024;
    d2* taus = reinterpret_cast<d2*>(tk);
    double* th = tk + 64;
    // ---- H into registers (zero outside n x n)
    d2 a[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const int c = c0 + t;
        const d2 v = i <= c ? T0[up_idx(i, c)] : conj_d2(T0[up_idx(c, i)]);
        a[t] = (i < n && c < n) ? v : zero;
    }
    sync();
    if (lane == 0) {
        VB[TK_ONE] = one;
        VB[TK_ZERO] = zero;
    }
    // ---- tridiagonalisation: step k annihilates A[k+2.., k] with I - tau v v^H (v[k+1] = 1)
    int off = 0;
    for (int k = 0; k + 1 < n; ++k) {
        if (i == k) {
#pragma unroll
            for (int t = 0; t < 16; ++t) rowb[c0 + t] = a[t];
        }
        sync();
        const d2 x = (i > k && i < n) ? conj_d2(rowb[i]) : zero;   // A[i][k]
        const double ar = readlane_d(x.x, k + 1), ai = readlane_d(x.y, k + 1);
        const double xn2 = hsum32(i > k + 1 ? cabs2(x) : 0.0);
        d2 tau = zero, sc = zero;
        double beta = ar;
        if (xn2 > 0.0 || ai != 0.0) {   // zlarfg
            beta = -copysign(sqrt(fma(ar, ar, fma(ai, ai, xn2))), ar);
            tau = make_double2((beta - ar) / beta, -ai / beta);
            const double dr = ar - beta, den = dr * dr + ai * ai;
            sc = make_double2(dr / den, -ai / den);   // 1 / (alpha - beta)
        }
        const d2 v = i == k + 1 ? one : (i > k + 1 ? cmul(x, sc) : zero);
        if (lane == 0) {
            dd[k] = rowb[k].x;
            ee[k + 1] = beta;
            e2[k + 1] = beta * beta;
            taus[k] = tau;
        }
        if (h == 0) {
            vsh[i] = v;
            if (i > k + 1 && i < n) VB[off + i - k - 2] = v;
        }
        off += n - k - 2;
        sync();
        if (tau.x != 0.0 || tau.y != 0.0) {
            // p = tau A v over the trailing block (v vanishes elsewhere), w = p - (tau / 2) (p^H v) v
            d2 pa = zero;
#pragma unroll
            for (int t = 0; t < 16; ++t) pa = cadd(pa, cmul(a[t], vsh[c0 + t]));
            pa.x = xor32_sum(pa.x);
            pa.y = xor32_sum(pa.y);
            const d2 p = i > k ? cmul(tau, pa) : zero;
            const double pvr = hsum32(p.x * v.x + p.y * v.y), pvi = hsum32(p.x * v.y - p.y * v.x);
            const d2 al = cscale(cmul(tau, make_double2(pvr, pvi)), -0.5);
            const d2 w = cadd(p, cmul(al, v));
            if (h == 0) wsh[i] = w;
            sync();
            // A -= v w^H + w v^H (rows and columns <= k untouched: v and w vanish there)
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const d2 vc = vsh[c0 + t], wc = wsh[c0 + t];
                d2 nv = csub(a[t], cadd(cmul(v, conj_d2(wc)), cmul(w, conj_d2(vc))));
                if (c0 + t == i) nv.y = 0.0;
                a[t] = nv;
            }
        }
        sync();
    }
    if (i == n - 1) {
#pragma unroll
        for (int t = 0; t < 16; ++t) rowb[c0 + t] = a[t];
    }
    sync();
    if (lane == 0) {
        dd[n - 1] = rowb[n - 1].x;
        ee[0] = 0.0;
        e2[0] = 0.0;
    }
    sync();
    TK_STAMP();
    // ---- the K largest eigenvalues: G lanes per eigenvalue ej, two probes each, (2G + 1)-section per round
    double glo = INFINITY, ghi = -INFINITY;
    if (lane < n) {
        const double r = fabs(ee[lane]) + (lane + 1 < n ? fabs(ee[lane + 1]) : 0.0);
        glo = dd[lane] - r;
        ghi = dd[lane] + r;
    }
    glo = -wave_max(-glo);
    ghi = wave_max(ghi);
    const double scale = fmax(fabs(glo), fabs(ghi));
    if (!(scale > 1e-200 && scale < 1e200)) return false;
    const double tiny = 1e-46 * scale, tol = 0x1p-51 * scale;
    const int G = 64 / K, ej = lane / G, pq = lane - ej * G;
    const bool act = ej < K;
    const double nsec = (double)(2 * G + 1);
    double lo = glo, hi = ghi;
    for (int round = 0; round < 48; ++round) {
        if (!__any(act && hi - lo > tol)) break;
        const double stp = (hi - lo) / nsec;
        const double x0 = lo + stp * (double)(2 * pq + 1), x1 = lo + stp * (double)(2 * pq + 2);
        double d0 = dd[0] - x0, d1 = dd[0] - x1;
        if (fabs(d0) < tiny) d0 = -tiny;
        if (fabs(d1) < tiny) d1 = -tiny;
        int n0 = d0 < 0.0, n1 = d1 < 0.0;
#pragma unroll
        for (int j = 1; j < ZT; ++j) {   // (unrolled: the LDS loads issue ahead of the chains)
            const double dj = dd[j], q2 = e2[j];
            double u0 = (dj - x0) - q2 * frcp(d0), u1 = (dj - x1) - q2 * frcp(d1);
            if (fabs(u0) < tiny) u0 = -tiny;
            if (fabs(u1) < tiny) u1 = -tiny;
            const bool in = j < n;
            d0 = in ? u0 : d0;
            d1 = in ? u1 : d1;
            n0 += in && u0 < 0.0;
            n1 += in && u1 < 0.0;
        }
        // eigenvalue ej (descending) lies above x iff at least ej + 1 eigenvalues are >= x
        double nlo = lo, nhi = hi;
        if (n - n0 >= ej + 1) nlo = x0;
        if (n - n1 >= ej + 1) nlo = x1;
        if (n - n1 <= ej) nhi = x1;
        if (n - n0 <= ej) nhi = x0;
        for (int t = 0; t < G; ++t) {   // combine the eigenvalue's G lanes
            const int src = (ej * G + t) & 63;
            nlo = fmax(nlo, __shfl(nlo, src, 64));
            nhi = fmin(nhi, __shfl(nhi, src, 64));
        }
        if (act) {
            lo = nlo;
            hi = nhi;
        }
    }
    const double thv = 0.5 * (lo + hi);
    if (act && pq == 0) th[ej] = thv;
    TK_STAMP();
    // ---- their vectors: twisted factorisation at theta (lane ej G)
    if (act && pq == 0) {
        double* dp = S + ej * TK_LD;
        double* dm = dp + 32;
        for (int j = 0; j < n; ++j) {
            const double d = (dd[j] - thv) - (j > 0 ? e2[j] / dp[j - 1] : 0.0);
            dp[j] = d == 0.0 ? tiny : d;
        }
        for (int j = n - 1; j >= 0; --j) {
            const double d = (dd[j] - thv) - (j + 1 < n ? e2[j + 1] / dm[j + 1] : 0.0);
            dm[j] = d == 0.0 ? tiny : d;
        }
        int r = 0;
        double gb = INFINITY;
        for (int j = 0; j < n; ++j) {
            const double g = fabs(dp[j] + dm[j] - (dd[j] - thv));
            if (g < gb) {
                gb = g;
                r = j;
            }
        }
        double nrm = 1.0, sv = 1.0;
        for (int j = r - 1; j >= 0; --j) {
            sv = -ee[j + 1] * sv / dp[j];
            dp[j] = sv;
            nrm += sv * sv;
        }
        sv = 1.0;
        for (int j = r + 1; j < n; ++j) {
            sv = -ee[j] * sv / dm[j];
            dp[j] = sv;
            nrm += sv * sv;
        }
        dp[r] = 1.0;
        const double inv = 1.0 / sqrt(nrm);
        for (int j = 0; j < 32; ++j) dp[j] = j < n ? dp[j] * inv : 0.0;
    }
    sync();
    TK_STAMP();
    // ---- Householder QR of [s_0 .. s_{K-1}]: column j becomes u_j (explicit: 0 above j, 1 at j), tau_j at + 32
    for (int j = 0; j < K; ++j) {
        double* cj = S + j * TK_LD;
        const double xv = cj[i];
        const double a0 = cj[j];
        const double sig = hsum32((i > j && i < n) ? xv * xv : 0.0);
        double tq = 0.0, iv = 0.0;
        if (sig > 0.0) {
            const double bt = -copysign(sqrt(fma(a0, a0, sig)), a0);
            tq = (bt - a0) / bt;
            iv = 1.0 / (a0 - bt);
        }
        const double u = i < j ? 0.0 : (i == j ? 1.0 : (i < n ? xv * iv : 0.0));
        sync();
        if (h == 0) cj[i] = u;
        if (lane == 0) cj[32] = tq;
        if (tq != 0.0) {
            for (int cb = j + 1; cb < K; cb += 2) {   // half h takes column cb + h
                const int c = cb + h;
                double* cc = S + min(c, K - 1) * TK_LD;
                const double dot = hsum32(c < K ? u * cc[i] : 0.0);
                if (c < K && i >= j) cc[i] -= tq * u * dot;
            }
        }
        sync();
    }
    TK_STAMP();
    // ---- Q_s = H_0 .. H_{K-1} I: lane (column i, rows 16 h ..)
    double q[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) q[t] = (c0 + t == i) ? 1.0 : 0.0;
    for (int j = K - 1; j >= 0; --j) {
        const double* cj = S + j * TK_LD;
        const double tq = cj[32];
        double dot = 0.0;
#pragma unroll
        for (int t = 0; t < 16; ++t) dot += cj[c0 + t] * q[t];
        dot = xor32_sum(dot);
        const double td = tq * dot;
#pragma unroll
        for (int t = 0; t < 16; ++t) q[t] -= cj[c0 + t] * td;
    }
    TK_STAMP();
    // ---- the Ritz residuals of columns 0..K-1 against T
    {
        const double tht = i < K ? th[i] : 0.0;
        const double nb = __shfl_xor(h ? q[0] : q[15], 32, 64);   // the row across the halves' boundary
        double r2 = 0.0;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int r = c0 + t;
            const double qm = t > 0 ? q[t - 1] : (h ? nb : 0.0);
            const double qp = t < 15 ? q[t + 1] : (h ? 0.0 : nb);
            const double rv = (dd[r] - tht) * q[t] + (r > 0 ? ee[r] * qm : 0.0) + (r + 1 < n ? ee[r + 1] * qp : 0.0);
            r2 += r < n ? rv * rv : 0.0;
        }
        r2 = xor32_sum(r2);
        const double lim = 0x1p-44 * scale;
        if (__any(i < K && !(r2 <= lim * lim))) return false;
    }
    // ---- R = Q_h Q_s: the tridiagonalisation's reflectors, last first
    d2 qc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) qc[t] = make_double2(q[t], 0.0);
    for (int k = n - 2; k >= 0; --k) {
        const d2 tau = taus[k];
        if (tau.x == 0.0 && tau.y == 0.0) continue;
        const int o = k * (n - 2) - k * (k - 1) / 2 - k - 2;   // VB index of row r: o + r (r in (k+1, n))
        auto vidx = [&](int r) { return (r > k + 1 && r < n) ? o + r : (r == k + 1 ? TK_ONE : TK_ZERO); };
        d2 dot = zero;
#pragma unroll
        for (int t = 0; t < 16; ++t) dot = cadd(dot, cmulc(VB[vidx(c0 + t)], qc[t]));
        dot.x = xor32_sum(dot.x);
        dot.y = xor32_sum(dot.y);
        const d2 td = cmul(tau, dot);
#pragma unroll
        for (int t = 0; t < 16; ++t) qc[t] = csub(qc[t], cmul(VB[vidx(c0 + t)], td));
    }
    sync();   // every lane is done with VB and S
#pragma unroll
    for (int t = 0; t < 16; ++t) T0[(c0 + t) * ZHS + i] = qc[t];
    sync();
#ifdef ACE_DEBUG_TK
    TK_STAMP();
    if (lane == 0 && (blockIdx.x == 5 || blockIdx.x == 1500))
        printf("tk b %d: tri %llu bis %llu twist %llu qr %llu qs %llu res+bt %llu (x10ns)\n", (int)blockIdx.x, tkt[1] - tkt[0],
               tkt[2] - tkt[1], tkt[3] - tkt[2], tkt[4] - tkt[3], tkt[5] - tkt[4], tkt[6] - tkt[5]);
#endif
#undef TK_STAMP
    return true;
}

}  // namespace
}  // namespace ace
