// Downstream beamformer: batched svd_beamformer /
// svd_beamformer_compensation (reference main/codebook_library.py:57-138), the consumer
// of recovered channels in codebook_generator (:192-213).
//
// Per realisation: Vh of zgesdd(H) and of zgesdd(H^T) (JOBZ='A', LAPACK's phase and sign
// convention, because the beam codes quantise those phases), 2-bit phase quantisation,
// the all-pairs received-power search |wt_i^T H wr_j|^2 with first-argmax, and the code
// strings of the winning pair.  One wavefront per realisation, everything in LDS:
//
//   zgebd2     Householder bidiagonalisation (zlarfg conventions), lane = column / row
//   dbdsqr     implicit-shift / zero-shift QR on the real bidiagonal; the scalar recurrence
//              runs redundantly in every lane (uniform control flow, no broadcasts), each
//              lane applies the rotations to its own column of VT as they are generated
//   zunmbr     Vh = VT * P^H, reflectors applied right-to-left, lane = row
//   search     T = H wr (exact +-1/+-j multipliers), M = wt^T T, argmax over lanes
//
// For n <= 25 this is zgesdd's path (dbdsdc -> dlasdq -> dbdsqr).  For 26..32 numpy's
// zgesdd uses divide and conquer (dlasd0: two dlasdq leaves and one dlasd1 merge), whose real
// singular vectors equal dbdsqr's up to sign; the merge's sign convention is applied after
// dbdsqr (gesdd_vh).  The status bit ACE_ST_BF_DC marks those realisations: a vector the merge
// deflated (the null space of a rank-deficient H) can still differ from numpy's.
#include "ace_common.hpp"
#include "ace_host.hpp"

// No a*b+c -> fma contraction in this file: LAPACK (numpy's scipy-openblas build) evaluates
// dbdsqr's recurrences unfused, and with a converged (perfect) shift the bottom rotation of a
// chase is a cancellation whose rounding decides the sign of a singular vector -- i.e. a
// code bit.  Fused rounding flips it on ~1% of 16x16 matrices.
#pragma clang fp contract(off)

namespace ace {
namespace {

constexpr int BF_NMAX = 32;
constexpr int BF_SMLSIZ = 25;  // ilaenv(9) — dbdsdc's switch to divide and conquer
constexpr double kEps = 0x1p-53;
constexpr double kSafmin = 0x1p-1022;
constexpr double kSafmax = 0x1p+1022;
constexpr double kHalfPi = 1.5707963267948966;  // numpy's np.pi / 2

// dbdsqr TOL = max(10, min(100, eps^(-1/8))) * eps
__device__ __forceinline__ double bd_tol() { return fmax(10.0, fmin(100.0, pow(kEps, -0.125))) * kEps; }

// Reference-LAPACK 3.10+ dlartg: c >= 0, r carries the sign of f.
__device__ __forceinline__ void dlartg(double f, double g, double& c, double& s, double& r) {
    const double rtmin = 0x1p-511, rtmax = 0x1.6a09e667f3bcdp+510;  // sqrt(safmin), sqrt(safmax/2)
    if (g == 0.0) { c = 1.0; s = 0.0; r = f; return; }
    if (f == 0.0) { c = 0.0; s = copysign(1.0, g); r = fabs(g); return; }
    const double f1 = fabs(f), g1 = fabs(g);
    if (f1 > rtmin && f1 < rtmax && g1 > rtmin && g1 < rtmax) {
        const double d = sqrt(f * f + g * g);
        c = f1 / d;
        r = copysign(d, f);
        s = g / r;
    } else {
        const double u = fmin(kSafmax, fmax(kSafmin, fmax(f1, g1)));
        const double fs = f / u, gs = g / u, d = sqrt(fs * fs + gs * gs);
        c = fabs(fs) / d;
        r = copysign(d, f);
        s = gs / r;
        r *= u;
    }
}

// LAPACK dlas2: smaller singular value of [[f, g], [0, h]] (the shift).
__device__ double dlas2_min(double f, double g, double h) {
    const double fa = fabs(f), ga = fabs(g), ha = fabs(h);
    const double fhmn = fmin(fa, ha), fhmx = fmax(fa, ha);
    if (fhmn == 0.0) return 0.0;
    if (ga < fhmx) {
        const double as = 1.0 + fhmn / fhmx, at = (fhmx - fhmn) / fhmx, au = (ga / fhmx) * (ga / fhmx);
        const double c = 2.0 / (sqrt(as * as + au) + sqrt(at * at + au));
        return fhmn * c;
    }
    const double au = fhmx / ga;
    if (au == 0.0) return (fhmn * fhmx) / ga;
    const double as = 1.0 + fhmn / fhmx, at = (fhmx - fhmn) / fhmx;
    const double c = 1.0 / (sqrt(1.0 + (as * au) * (as * au)) + sqrt(1.0 + (at * au) * (at * au)));
    const double ssmin = (fhmn * c) * au;
    return ssmin + ssmin;
}

// LAPACK dlasv2: SVD of [[f, g], [0, h]].
__device__ void dlasv2(double f, double g, double h, double& ssmin, double& ssmax, double& snr, double& csr,
                       double& snl, double& csl) {
    double ft = f, fa = fabs(f), ht = h, ha = fabs(h);
    int pmax = 1;
    const bool swap = ha > fa;
    if (swap) {
        pmax = 3;
        double t = ft; ft = ht; ht = t;
        t = fa; fa = ha; ha = t;
    }
    const double gt = g, ga = fabs(g);
    double clt, crt, slt, srt;
    if (ga == 0.0) {
        ssmin = ha; ssmax = fa;
        clt = 1.0; crt = 1.0; slt = 0.0; srt = 0.0;
    } else {
        bool gasmal = true;
        if (ga > fa) {
            pmax = 2;
            if (fa / ga < kEps) {
                gasmal = false;
                ssmax = ga;
                ssmin = ha > 1.0 ? fa / (ga / ha) : (fa / ga) * ha;
                clt = 1.0; slt = ht / gt; srt = 1.0; crt = ft / gt;
            }
        }
        if (gasmal) {
            const double d = fa - ha;
            double l = (d == fa) ? 1.0 : d / fa;
            const double m = gt / ft;
            double t = 2.0 - l;
            const double mm = m * m, tt = t * t, s = sqrt(tt + mm);
            const double r = (l == 0.0) ? fabs(m) : sqrt(l * l + mm);
            const double a = 0.5 * (s + r);
            ssmin = ha / a;
            ssmax = fa * a;
            if (mm == 0.0) {
                if (l == 0.0) t = copysign(2.0, ft) * copysign(1.0, gt);
                else t = gt / copysign(d, ft) + m / t;
            } else {
                t = (m / (s + t) + m / (r + l)) * (1.0 + a);
            }
            l = sqrt(t * t + 4.0);
            crt = 2.0 / l;
            srt = t / l;
            clt = (crt + srt * m) / a;
            slt = (ht / ft) * srt / a;
        }
    }
    if (swap) { csl = srt; snl = crt; csr = slt; snr = clt; }
    else { csl = clt; snl = slt; csr = crt; snr = srt; }
    double tsign;
    if (pmax == 1) tsign = copysign(1.0, csr) * copysign(1.0, csl) * copysign(1.0, f);
    else if (pmax == 2) tsign = copysign(1.0, snr) * copysign(1.0, csl) * copysign(1.0, g);
    else tsign = copysign(1.0, snr) * copysign(1.0, snl) * copysign(1.0, h);
    ssmax = copysign(ssmax, tsign);
    ssmin = copysign(ssmin, tsign * copysign(1.0, f) * copysign(1.0, h));
}

// LAPACK dlapy3
__device__ __forceinline__ double dlapy3(double x, double y, double z) {
    const double xa = fabs(x), ya = fabs(y), za = fabs(z), w = fmax(xa, fmax(ya, za));
    if (w == 0.0 || w > 1.79e308) return xa + ya + za;
    const double a = xa / w, b = ya / w, c = za / w;
    return w * sqrt(a * a + b * b + c * c);
}

// zlarfg on (alpha, x) with ||x|| = xnorm: beta (real), tau, and the scale for x.
__device__ __forceinline__ void zlarfg(d2 alpha, double xnorm, double& beta, d2& tau, d2& scal) {
    const double ar = alpha.x, ai = alpha.y;
    if (xnorm == 0.0 && ai == 0.0) {
        beta = ar;
        tau = make_double2(0.0, 0.0);
        scal = make_double2(1.0, 0.0);
        return;
    }
    beta = -copysign(dlapy3(ar, ai, xnorm), ar);
    tau = make_double2((beta - ar) / beta, -ai / beta);
    const d2 den = make_double2(ar - beta, ai);  // zladiv(1, alpha - beta)
    const double q = den.x * den.x + den.y * den.y;
    scal = make_double2(den.x / q, -den.y / q);
}

__device__ __forceinline__ d2 cconj(d2 a) { return make_double2(a.x, -a.y); }

struct BfShared {  // per-wave LDS carve (one realisation per block)
    d2* A;       // [n][ld] working matrix / reflector storage, later H
    d2* X;       // [n][ld] VT (real parts) then Vh, later T = H wr
    double* d;   // [BF_NMAX] bidiagonal
    double* e;   // [BF_NMAX]
    d2* taup;    // [BF_NMAX]
    d2* Q;       // [N][ld] zgelq2's H(1) ... H(m) (tx != rx only)
    signed char* qr;  // [rx][rx] quantised phases of Vh(H)   (around(angle/(pi/2)), -2..2)
    signed char* qt;  // [tx][tx] quantised phases of Vh(H^T)
};

__device__ __forceinline__ void wsync() { __syncthreads(); }  // block == one wavefront

// zgebd2 for m >= n (upper bidiagonal d [n], e [n - 1]) of the m x n matrix in sh.A: the column reflectors'
// tails stay below the diagonal, G(i) (i < n - 1) acts on columns i + 1 .. n - 1 with its tail in A[i][i + 2 ..]
__device__ void zgebd2_upper(const BfShared& sh, int m, int n, int ld, int lane) {
    d2* A = sh.A;
    double* dd = sh.d;
    double* ee = sh.e;
    for (int i = 0; i < n; ++i) {
        // column reflector H(i) annihilating A(i+1:n, i)
        double part = 0.0;
        if (lane > i && lane < m) part = cabs2(A[lane * ld + i]);
        const double xnorm = sqrt(wave_sum(part));
        double beta;
        d2 tauq, scal;
        zlarfg(A[i * ld + i], xnorm, beta, tauq, scal);
        wsync();
        if (lane > i && lane < m) A[lane * ld + i] = cmul(A[lane * ld + i], scal);
        dd[i] = beta;
        wsync();
        if (i < n - 1) {
            // A(i:n, i+1:n) := H(i)^H A(i:n, i+1:n); lane = column
            if (lane > i && lane < n) {
                const int c = lane;
                d2 w = A[i * ld + c];
                for (int r = i + 1; r < m; ++r) w = cadd(w, cmulc(A[r * ld + i], A[r * ld + c]));
                const d2 tw = cmul(cconj(tauq), w);
                A[i * ld + c] = csub(A[i * ld + c], tw);
                for (int r = i + 1; r < m; ++r) A[r * ld + c] = csub(A[r * ld + c], cmul(A[r * ld + i], tw));
            }
            wsync();
            // row reflector G(i) annihilating A(i, i+2:n) (on the conjugated row)
            double p2 = 0.0;
            if (lane > i + 1 && lane < n) p2 = cabs2(A[i * ld + lane]);
            const double xn2 = sqrt(wave_sum(p2));
            double beta2;
            d2 taup, scal2;
            zlarfg(cconj(A[i * ld + i + 1]), xn2, beta2, taup, scal2);
            wsync();
            if (lane > i + 1 && lane < n) A[i * ld + lane] = cmul(cconj(A[i * ld + lane]), scal2);  // v tail
            ee[i] = beta2;
            sh.taup[i] = taup;
            wsync();
            // A(i+1:m, i+1:n) := A G(i), G = I - taup v v^H; lane = row
            if (lane > i && lane < m) {
                const int r = lane;
                d2 w = A[r * ld + i + 1];
                for (int c = i + 2; c < n; ++c) w = cadd(w, cmul(A[r * ld + c], A[i * ld + c]));
                const d2 tw = cmul(taup, w);
                A[r * ld + i + 1] = csub(A[r * ld + i + 1], tw);
                for (int c = i + 2; c < n; ++c) A[r * ld + c] = csub(A[r * ld + c], cmul(tw, cconj(A[i * ld + c])));
            }
            wsync();
        }
    }
}

// Right singular vectors of the real upper bidiagonal (sh.d, sh.e) of order n into VT = sh.X [nc][nc] (nc >= n:
// rows and columns >= n stay the identity's), zgesdd's sign convention included.  Returns false when dbdsqr
// exhausted its iteration budget.
__device__ bool bd_vt(const BfShared& sh, int n, int nc, int ld, int lane) {
    d2* X = sh.X;
    double* dd = sh.d;
    double* ee = sh.e;
    // ---------------- VT := I (real parts of X)
    if (lane < nc)
        for (int r = 0; r < nc; ++r) X[r * ld + lane] = make_double2(r == lane ? 1.0 : 0.0, 0.0);
    wsync();
    bool ok = true;
    // divide and conquer (n > 25): the bidiagonal's row n / 2 (dlasdt's root, dlasd0's merge row) before dbdsqr
    // overwrites it
    const int mid = n / 2;
    const double dmid = n > BF_SMLSIZ ? dd[mid] : 0.0, emid = n > BF_SMLSIZ ? ee[mid] : 0.0;
    if (n > 1) {
        // ---------------- dbdsqr (ncvt = n, relative accuracy); 1-based m/ll as in LAPACK
        const double tol = bd_tol();
        const bool col = lane < nc;
        auto rot = [&](int i, double c, double s) {  // drot on VT rows i, i+1 (0-based)
            if (col) {
                const double x = X[i * ld + lane].x, y = X[(i + 1) * ld + lane].x;
                X[i * ld + lane].x = c * x + s * y;
                X[(i + 1) * ld + lane].x = c * y - s * x;
            }
        };
        double smax = 0.0;
        for (int i = 0; i < n; ++i) smax = fmax(smax, fabs(dd[i]));
        for (int i = 0; i < n - 1; ++i) smax = fmax(smax, fabs(ee[i]));
        double sminoa = fabs(dd[0]);
        if (sminoa != 0.0) {
            double mu = sminoa;
            for (int i = 1; i < n; ++i) {
                mu = fabs(dd[i]) * (mu / (mu + fabs(ee[i - 1])));
                sminoa = fmin(sminoa, mu);
                if (sminoa == 0.0) break;
            }
        }
        sminoa = sminoa / sqrt((double)n);
        const double thresh = fmax(tol * sminoa, 6.0 * (n * (n * kSafmin)));
        const int maxitdivn = 6 * n;
        int iterdivn = 0, iter = -1, oldll = -1, oldm = -1, idir = 0;
        int m = n;
        double sminl = 0.0;
        while (m > 1) {
            if (iter >= n) {
                iter -= n;
                if (++iterdivn >= maxitdivn) { ok = false; break; }
            }
            smax = fabs(dd[m - 1]);
            int ll = 0;
            bool split = false;
            for (int lll = 1; lll < m; ++lll) {
                ll = m - lll;
                const double abss = fabs(dd[ll - 1]), abse = fabs(ee[ll - 1]);
                if (abse <= thresh) { split = true; break; }
                smax = fmax(smax, fmax(abss, abse));
            }
            if (split) {
                ee[ll - 1] = 0.0;
                if (ll == m - 1) { m -= 1; continue; }
            } else {
                ll = 0;
            }
            ll += 1;
            if (ll == m - 1) {  // 2 x 2 block
                double ssmin, ssmax, sinr, cosr, sinl, cosl;
                dlasv2(dd[m - 2], ee[m - 2], dd[m - 1], ssmin, ssmax, sinr, cosr, sinl, cosl);
                dd[m - 2] = ssmax;
                ee[m - 2] = 0.0;
                dd[m - 1] = ssmin;
                rot(m - 2, cosr, sinr);
                m -= 2;
                continue;
            }
            if (ll > oldm || m < oldll) idir = fabs(dd[ll - 1]) >= fabs(dd[m - 1]) ? 1 : 2;
            bool conv = false;
            if (idir == 1) {
                if (fabs(ee[m - 2]) <= tol * fabs(dd[m - 1])) { ee[m - 2] = 0.0; continue; }
                double mu = fabs(dd[ll - 1]);
                sminl = mu;
                for (int lll = ll; lll < m; ++lll) {
                    if (fabs(ee[lll - 1]) <= tol * mu) { ee[lll - 1] = 0.0; conv = true; break; }
                    mu = fabs(dd[lll]) * (mu / (mu + fabs(ee[lll - 1])));
                    sminl = fmin(sminl, mu);
                }
            } else {
                if (fabs(ee[ll - 1]) <= tol * fabs(dd[ll - 1])) { ee[ll - 1] = 0.0; continue; }
                double mu = fabs(dd[m - 1]);
                sminl = mu;
                for (int lll = m - 1; lll >= ll; --lll) {
                    if (fabs(ee[lll - 1]) <= tol * mu) { ee[lll - 1] = 0.0; conv = true; break; }
                    mu = fabs(dd[lll - 1]) * (mu / (mu + fabs(ee[lll - 1])));
                    sminl = fmin(sminl, mu);
                }
            }
            if (conv) continue;
            oldll = ll;
            oldm = m;
            double shift;
            if (n * tol * (sminl / smax) <= fmax(kEps, 0.01 * tol)) {
                shift = 0.0;
            } else {
                double sll;
                if (idir == 1) { sll = fabs(dd[ll - 1]); shift = dlas2_min(dd[m - 2], ee[m - 2], dd[m - 1]); }
                else { sll = fabs(dd[m - 1]); shift = dlas2_min(dd[ll - 1], ee[ll - 1], dd[ll]); }
                if (sll > 0.0 && (shift / sll) * (shift / sll) < kEps) shift = 0.0;
            }
            iter += m - ll;
            if (shift == 0.0) {
                double cs = 1.0, sn, r, oldcs = 1.0, oldsn = 0.0;
                if (idir == 1) {
                    for (int i = ll; i < m; ++i) {
                        dlartg(dd[i - 1] * cs, ee[i - 1], cs, sn, r);
                        if (i > ll) ee[i - 2] = oldsn * r;
                        double dn;
                        dlartg(oldcs * r, dd[i] * sn, oldcs, oldsn, dn);
                        dd[i - 1] = dn;
                        rot(i - 1, cs, sn);
                    }
                    const double h = dd[m - 1] * cs;
                    dd[m - 1] = h * oldcs;
                    ee[m - 2] = h * oldsn;
                    if (fabs(ee[m - 2]) <= thresh) ee[m - 2] = 0.0;
                } else {
                    for (int i = m; i > ll; --i) {
                        dlartg(dd[i - 1] * cs, ee[i - 2], cs, sn, r);
                        if (i < m) ee[i - 1] = oldsn * r;
                        double dn;
                        dlartg(oldcs * r, dd[i - 2] * sn, oldcs, oldsn, dn);
                        dd[i - 1] = dn;
                        rot(i - 2, oldcs, -oldsn);
                    }
                    const double h = dd[ll - 1] * cs;
                    dd[ll - 1] = h * oldcs;
                    ee[ll - 1] = h * oldsn;
                    if (fabs(ee[ll - 1]) <= thresh) ee[ll - 1] = 0.0;
                }
            } else {
                double cosr, sinr, cosl, sinl, r;
                if (idir == 1) {
                    double f = (fabs(dd[ll - 1]) - shift) * (copysign(1.0, dd[ll - 1]) + shift / dd[ll - 1]);
                    double g = ee[ll - 1];
                    for (int i = ll; i < m; ++i) {
                        dlartg(f, g, cosr, sinr, r);
                        if (i > ll) ee[i - 2] = r;
                        f = cosr * dd[i - 1] + sinr * ee[i - 1];
                        ee[i - 1] = cosr * ee[i - 1] - sinr * dd[i - 1];
                        g = sinr * dd[i];
                        dd[i] = cosr * dd[i];
                        dlartg(f, g, cosl, sinl, r);
                        dd[i - 1] = r;
                        f = cosl * ee[i - 1] + sinl * dd[i];
                        dd[i] = cosl * dd[i] - sinl * ee[i - 1];
                        if (i < m - 1) {
                            g = sinl * ee[i];
                            ee[i] = cosl * ee[i];
                        }
                        rot(i - 1, cosr, sinr);
                    }
                    ee[m - 2] = f;
                    if (fabs(ee[m - 2]) <= thresh) ee[m - 2] = 0.0;
                } else {
                    double f = (fabs(dd[m - 1]) - shift) * (copysign(1.0, dd[m - 1]) + shift / dd[m - 1]);
                    double g = ee[m - 2];
                    for (int i = m; i > ll; --i) {
                        dlartg(f, g, cosr, sinr, r);
                        if (i < m) ee[i - 1] = r;
                        f = cosr * dd[i - 1] + sinr * ee[i - 2];
                        ee[i - 2] = cosr * ee[i - 2] - sinr * dd[i - 1];
                        g = sinr * dd[i - 2];
                        dd[i - 2] = cosr * dd[i - 2];
                        dlartg(f, g, cosl, sinl, r);
                        dd[i - 1] = r;
                        f = cosl * ee[i - 2] + sinl * dd[i - 2];
                        dd[i - 2] = cosl * dd[i - 2] - sinl * ee[i - 2];
                        if (i > ll + 1) {
                            g = sinl * ee[i - 3];
                            ee[i - 3] = cosl * ee[i - 3];
                        }
                        rot(i - 2, cosl, -sinl);
                    }
                    ee[ll - 1] = f;
                    if (fabs(ee[ll - 1]) <= thresh) ee[ll - 1] = 0.0;
                }
            }
        }
        wsync();
        // make singular values positive; selection sort into decreasing order
        for (int i = 0; i < n; ++i)
            if (dd[i] < 0.0) {
                dd[i] = -dd[i];
                if (col) X[i * ld + lane].x = -X[i * ld + lane].x;
            }
        for (int i = 1; i < n; ++i) {
            int isub = 1;
            double smin = dd[0];
            for (int j = 2; j <= n + 1 - i; ++j)
                if (dd[j - 1] <= smin) { isub = j; smin = dd[j - 1]; }
            const int last = n + 1 - i;
            if (isub != last) {
                dd[isub - 1] = dd[last - 1];
                dd[last - 1] = smin;
                if (col) {
                    const double t = X[(isub - 1) * ld + lane].x;
                    X[(isub - 1) * ld + lane].x = X[(last - 1) * ld + lane].x;
                    X[(last - 1) * ld + lane].x = t;
                }
            }
        }
        wsync();
        if (n > BF_SMLSIZ && lane < n) {
            // zgesdd's dbdsdc (n > SMLSIZ = 25) -> dlasd0: one merge at row mid of the leaves [0, mid) (dlasdq on
            // mid x (mid + 1)) and (mid, n) (dlasdq on the rest), dlasd1 -> dlasd3 builds every non-deflated left
            // vector with its merge-row component -1 / ||.|| (dlasd3: U(1, i) = -1, the first deflated coordinate being
            // that row).  The vectors equal dbdsqr's up to sign, so row i of VT flips where u_i(mid) =
            // (d_mid v_i(mid) + e_mid v_i(mid + 1)) / s_i > 0.  Deflated vectors (z_j below 64 eps: a subproblem
            // vector with no merge-row component, e.g. the null space of an exactly rank-deficient H) keep the sign
            // of the leaf's own dbdsqr, which is not reproduced (nor is the basis of a degenerate null space): those
            // are what ACE_ST_BF_DC still flags
            const int r = lane;
            const double um = dmid * X[r * ld + mid].x + emid * X[r * ld + mid + 1].x;
            if (um > 0.0)
                for (int c = 0; c < n; ++c) X[r * ld + c].x = -X[r * ld + c].x;
        }
        wsync();
    }
    return ok;
}

// Vh := VT P^H = VT G(k-1)^H ... G(0)^H on VT = sh.X [nc][nc]; G(i) acts on columns c0 = i + off .. nc - 1 with
// the leading 1 at c0 and its tail in A[i][c0 + 1 ..] (off = 1: zgebd2 upper, 0: lower); lane = row
__device__ void apply_ph(const BfShared& sh, int nc, int k, int off, int ld, int lane) {
    const d2* A = sh.A;
    d2* X = sh.X;
    if (lane < nc) {
        const int r = lane;
        for (int i = k - 1; i >= 0; --i) {
            const int c0 = i + off;
            const d2 ctp = cconj(sh.taup[i]);
            d2 w = X[r * ld + c0];
            for (int c = c0 + 1; c < nc; ++c) w = cadd(w, cmul(X[r * ld + c], A[i * ld + c]));
            const d2 tw = cmul(ctp, w);
            X[r * ld + c0] = csub(X[r * ld + c0], tw);
            for (int c = c0 + 1; c < nc; ++c) X[r * ld + c] = csub(X[r * ld + c], cmul(tw, cconj(A[i * ld + c])));
        }
    }
    wsync();
}

// zgebd2 for m < n (lower bidiagonal d [m], e [m - 1]): G(i) on the conjugated row A(i, i:n) (columns i .. n - 1,
// tail in A[i][i + 1 ..]), then H(i) annihilating A(i + 2:m, i)
__device__ void zgebd2_lower(const BfShared& sh, int m, int n, int ld, int lane) {
    d2* A = sh.A;
    double* dd = sh.d;
    double* ee = sh.e;
    for (int i = 0; i < m; ++i) {
        double p2 = 0.0;
        if (lane > i && lane < n) p2 = cabs2(A[i * ld + lane]);
        const double xn2 = sqrt(wave_sum(p2));
        double beta;
        d2 taup, scal;
        zlarfg(cconj(A[i * ld + i]), xn2, beta, taup, scal);
        wsync();
        if (lane > i && lane < n) A[i * ld + lane] = cmul(cconj(A[i * ld + lane]), scal);  // v tail
        dd[i] = beta;
        sh.taup[i] = taup;
        wsync();
        if (i == m - 1) break;
        // A(i+1:m, i:n) := A G(i); lane = row
        if (lane > i && lane < m) {
            const int r = lane;
            d2 w = A[r * ld + i];
            for (int c = i + 1; c < n; ++c) w = cadd(w, cmul(A[r * ld + c], A[i * ld + c]));
            const d2 tw = cmul(taup, w);
            A[r * ld + i] = csub(A[r * ld + i], tw);
            for (int c = i + 1; c < n; ++c) A[r * ld + c] = csub(A[r * ld + c], cmul(tw, cconj(A[i * ld + c])));
        }
        wsync();
        // H(i) annihilating A(i+2:m, i)
        double part = 0.0;
        if (lane > i + 1 && lane < m) part = cabs2(A[lane * ld + i]);
        const double xnorm = sqrt(wave_sum(part));
        double beta2;
        d2 tauq, scal2;
        zlarfg(A[(i + 1) * ld + i], xnorm, beta2, tauq, scal2);
        wsync();
        if (lane > i + 1 && lane < m) A[lane * ld + i] = cmul(A[lane * ld + i], scal2);
        ee[i] = beta2;
        wsync();
        // A(i+1:m, i+1:n) := H(i)^H A; lane = column
        if (lane > i && lane < n) {
            const int c = lane;
            d2 w = A[(i + 1) * ld + c];
            for (int r = i + 2; r < m; ++r) w = cadd(w, cmulc(A[r * ld + i], A[r * ld + c]));
            const d2 tw = cmul(cconj(tauq), w);
            A[(i + 1) * ld + c] = csub(A[(i + 1) * ld + c], tw);
            for (int r = i + 2; r < m; ++r) A[r * ld + c] = csub(A[r * ld + c], cmul(A[r * ld + i], tw));
        }
        wsync();
    }
}

// zgeqr2 (m > n): R in A[0:n][0:n], zero below the diagonal
__device__ void zgeqr2_r(const BfShared& sh, int m, int n, int ld, int lane) {
    d2* A = sh.A;
    for (int i = 0; i < n; ++i) {
        double part = 0.0;
        if (lane > i && lane < m) part = cabs2(A[lane * ld + i]);
        const double xnorm = sqrt(wave_sum(part));
        double beta;
        d2 tau, scal;
        zlarfg(A[i * ld + i], xnorm, beta, tau, scal);
        wsync();
        if (lane > i && lane < m) A[lane * ld + i] = cmul(A[lane * ld + i], scal);
        wsync();
        if (lane > i && lane < n) {  // A(i:m, i+1:n) := H(i)^H A; lane = column
            const int c = lane;
            d2 w = A[i * ld + c];
            for (int r = i + 1; r < m; ++r) w = cadd(w, cmulc(A[r * ld + i], A[r * ld + c]));
            const d2 tw = cmul(cconj(tau), w);
            A[i * ld + c] = csub(A[i * ld + c], tw);
            for (int r = i + 1; r < m; ++r) A[r * ld + c] = csub(A[r * ld + c], cmul(A[r * ld + i], tw));
        }
        wsync();
        if (lane == 0) A[i * ld + i] = make_double2(beta, 0.0);
        wsync();
    }
    if (lane < n)
        for (int r = lane + 1; r < n; ++r) A[r * ld + lane] = make_double2(0.0, 0.0);
    wsync();
}

// zgelq2 (m < n): L in A[0:m][0:m] (zero above the diagonal), sh.Q [n][n] := H(1) H(2) ... H(m), so that
// zunglq's Q = sh.Q^H (A = L Q[0:m])
__device__ void zgelq2_lq(const BfShared& sh, int m, int n, int ld, int lane) {
    d2* A = sh.A;
    d2* Qh = sh.Q;
    if (lane < n)
        for (int r = 0; r < n; ++r) Qh[r * ld + lane] = make_double2(r == lane ? 1.0 : 0.0, 0.0);
    for (int i = 0; i < m; ++i) {
        double p2 = 0.0;
        if (lane > i && lane < n) p2 = cabs2(A[i * ld + lane]);
        const double xn2 = sqrt(wave_sum(p2));
        double beta;
        d2 tau, scal;
        zlarfg(cconj(A[i * ld + i]), xn2, beta, tau, scal);
        wsync();
        if (lane > i && lane < n) A[i * ld + lane] = cmul(cconj(A[i * ld + lane]), scal);  // v tail
        wsync();
        // A(i+1:m, i:n) := A H(i) and Qh(:, i:n) := Qh H(i); lane = row
        if (lane > i && lane < m) {
            const int r = lane;
            d2 w = A[r * ld + i];
            for (int c = i + 1; c < n; ++c) w = cadd(w, cmul(A[r * ld + c], A[i * ld + c]));
            const d2 tw = cmul(tau, w);
            A[r * ld + i] = csub(A[r * ld + i], tw);
            for (int c = i + 1; c < n; ++c) A[r * ld + c] = csub(A[r * ld + c], cmul(tw, cconj(A[i * ld + c])));
        }
        if (lane < n) {
            const int r = lane;
            d2 w = Qh[r * ld + i];
            for (int c = i + 1; c < n; ++c) w = cadd(w, cmul(Qh[r * ld + c], A[i * ld + c]));
            const d2 tw = cmul(tau, w);
            Qh[r * ld + i] = csub(Qh[r * ld + i], tw);
            for (int c = i + 1; c < n; ++c) Qh[r * ld + c] = csub(Qh[r * ld + c], cmul(tw, cconj(A[i * ld + c])));
        }
        wsync();
        if (lane == 0) A[i * ld + i] = make_double2(beta, 0.0);
        wsync();
    }
    if (lane < m)
        for (int c = lane + 1; c < m; ++c) A[lane * ld + c] = make_double2(0.0, 0.0);
    wsync();
}

// Vh of zgesdd(JOBZ='A') for the square n x n matrix in sh.A, into sh.X
__device__ bool gesdd_vh_square(const BfShared& sh, int n, int ld, int lane) {
    zgebd2_upper(sh, n, n, ld, lane);
    if (n == 1) {
        if (lane == 0) sh.X[0] = make_double2(1.0, 0.0);  // dbdsdc n == 1: VT = 1
        wsync();
        return true;
    }
    const bool ok = bd_vt(sh, n, n, ld, lane);
    apply_ph(sh, n, n - 1, 1, ld, lane);
    return ok;
}

// Vh [n][n] of zgesdd(JOBZ='A') for the m x n matrix in sh.A, into sh.X (m, n <= 32), following zgesdd's
// path choice (MNTHR1 = INT(MINMN * 17 / 9)): QR first for m >= MNTHR1 (paths 1-4), LQ first for n >= MNTHR1
// (paths 1t-4t), the matrix itself otherwise (paths 5/6, 5t/6t: upper / lower bidiagonal)
template <bool RECT>
__device__ bool gesdd_vh(const BfShared& sh, int m, int n, int ld, int lane) {
    if constexpr (!RECT) return gesdd_vh_square(sh, n, ld, lane);   // (tx == rx: the square path alone)
    if (n == 1) {
        if (lane == 0) sh.X[0] = make_double2(1.0, 0.0);
        wsync();
        return true;
    }
    if (m == n) return gesdd_vh_square(sh, n, ld, lane);
    const int mnthr1 = (int)(min(m, n) * 17.0 / 9.0);
    if (m > n && m >= mnthr1) {
        zgeqr2_r(sh, m, n, ld, lane);
        return gesdd_vh_square(sh, n, ld, lane);
    }
    if (n > m && n >= mnthr1) {
        zgelq2_lq(sh, m, n, ld, lane);
        const bool ok = gesdd_vh_square(sh, m, ld, lane);
        // VT = [Vh_L Q[0:m]; Q[m:n]], Q = Qh^H; built in A, then copied to X; lane = column
        d2* A = sh.A;
        d2* X = sh.X;
        const d2* Qh = sh.Q;
        if (lane < n) {
            const int c = lane;
            for (int r = 0; r < m; ++r) {
                d2 acc = make_double2(0.0, 0.0);
                for (int k = 0; k < m; ++k) acc = cadd(acc, cmul(X[r * ld + k], cconj(Qh[c * ld + k])));
                A[r * ld + c] = acc;
            }
            for (int r = m; r < n; ++r) A[r * ld + c] = cconj(Qh[c * ld + r]);
        }
        wsync();
        if (lane < n)
            for (int r = 0; r < n; ++r) X[r * ld + lane] = A[r * ld + lane];
        wsync();
        return ok;
    }
    if (m > n) {
        zgebd2_upper(sh, m, n, ld, lane);
        const bool ok = bd_vt(sh, n, n, ld, lane);
        apply_ph(sh, n, n - 1, 1, ld, lane);
        return ok;
    }
    zgebd2_lower(sh, m, n, ld, lane);
    bool ok = true;
    if (m == 1) {
        if (lane < n)
            for (int r = 0; r < n; ++r) sh.X[r * ld + lane] = make_double2(r == lane ? 1.0 : 0.0, 0.0);
        wsync();
    } else {
        // dbdsdc('L'): rotate to upper bidiagonal on the left (the right vectors are unchanged); every lane runs
        // the scalar recurrence, lane 0 stores it
        double* dd = sh.d;
        double* ee = sh.e;
        double di = dd[0];
        for (int i = 0; i < m - 1; ++i) {
            double cs, sn, r;
            dlartg(di, ee[i], cs, sn, r);
            const double dn = dd[i + 1];
            wsync();
            if (lane == 0) {
                dd[i] = r;
                ee[i] = sn * dn;
            }
            di = cs * dn;
        }
        wsync();
        if (lane == 0) dd[m - 1] = di;
        wsync();
        ok = bd_vt(sh, m, n, ld, lane);
    }
    apply_ph(sh, n, m, 0, ld, lane);
    return ok;
}

// around(angle(z) / (pi/2)) in -2..2 (numpy's round-half-even == rint)
__device__ __forceinline__ signed char quant(d2 z) { return (signed char)rint(atan2(z.y, z.x) / kHalfPi); }

// z * j^k
__device__ __forceinline__ d2 rotk(d2 z, int k) {
    switch (k & 3) {
        case 0: return z;
        case 1: return make_double2(-z.y, z.x);
        case 2: return make_double2(-z.x, -z.y);
        default: return make_double2(z.y, -z.x);
    }
}

// argmax order: NaN first (numpy), then larger, ties -> smaller index
__device__ __forceinline__ bool bf_better(double a, int ia, double b, int ib) {
    const bool na = isnan(a), nb = isnan(b);
    if (na || nb) return na && (!nb || ia < ib);
    return a > b || (a == b && ia < ib);
}

// 2-bit code of exp(1j * -(q*pi/2)) * exp(-1j*off) (codebook_library.py:80-88, :122-127)
__device__ __forceinline__ unsigned char code_of(int q, bool has_off, double off) {
    const double th = -((double)q * kHalfPi);
    double re = cos(th), im = sin(th);
    if (has_off) {
        const double br = cos(off), bi = -sin(off);
        const double pr = re * br - im * bi, pi = re * bi + im * br;
        re = pr;
        im = pi;
    }
    double c = rint(atan2(im, re) / kHalfPi);
    if (c < 0) c += 4.0;
    if (c == 4.0) c = 0.0;
    return (unsigned char)c;
}

// RECT = false: tx == rx (the square path only, which keeps the kernel at four waves per SIMD)
template <bool RECT>
__global__ __launch_bounds__(64) void beamformer_kernel(int tx, int rx, const d2* __restrict__ H,
                                                        const double* __restrict__ offset,
                                                        unsigned char* __restrict__ wr_code,
                                                        unsigned char* __restrict__ wt_code, int32_t* __restrict__ beam_idx,
                                                        double* __restrict__ rss_out, uint32_t* __restrict__ status,
                                                        d2* __restrict__ vh_r, d2* __restrict__ vh_t) {
    extern __shared__ __align__(16) unsigned char bf_lds[];
    const int lane = threadIdx.x;
    const int N = max(tx, rx), ld = N + 1;
    const size_t b = blockIdx.x;
    const int nh = tx * rx;
    BfShared sh;
    sh.A = (d2*)bf_lds;
    sh.X = sh.A + N * ld;
    sh.Q = sh.X + N * ld;
    sh.taup = sh.Q + (tx != rx ? N * ld : 0);
    sh.d = (double*)(sh.taup + BF_NMAX);
    sh.e = sh.d + BF_NMAX;
    sh.qr = (signed char*)(sh.e + BF_NMAX);
    sh.qt = sh.qr + rx * rx;
    const d2* Hb = H + b * nh;

    // non-finite input: numpy's zgesdd fails (LinAlgError "SVD did not converge")
    bool bad = false;
    for (int k = lane; k < nh; k += 64) {
        const d2 h = Hb[k];
        bad |= !isfinite(h.x) || !isfinite(h.y);
    }
    uint32_t st = (min(tx, rx) > BF_SMLSIZ) ? ACE_ST_BF_DC : 0u;
    if (__any(bad)) {
        if (lane == 0) {
            status[b] = st | ACE_ST_BF_NONFINITE;
            beam_idx[2 * b] = -1;
            beam_idx[2 * b + 1] = -1;
            rss_out[b] = __builtin_nan("");
        }
        for (int k = lane; k < rx; k += 64) wr_code[b * rx + k] = 0;
        for (int k = lane; k < tx; k += 64) wt_code[b * tx + k] = 0;
        return;
    }
    bool ok = true;
    for (int pass = 0; pass < 2; ++pass) {
        // pass 0: zgesdd(H) [tx][rx] -> Vh [rx][rx] -> wr; pass 1: zgesdd(H^T) [rx][tx] -> [tx][tx] -> wt
        // (codebook_library.py:59-60)
        const int m = pass == 0 ? tx : rx, n = pass == 0 ? rx : tx;
        for (int k = lane; k < nh; k += 64) {
            const int r = k / rx, c = k - r * rx;   // H[r][c]
            if (pass == 0) sh.A[r * ld + c] = Hb[k];
            else sh.A[c * ld + r] = Hb[k];
        }
        wsync();
        ok &= gesdd_vh<RECT>(sh, m, n, ld, lane);
        signed char* q = pass == 0 ? sh.qr : sh.qt;
        d2* vh_out = pass == 0 ? vh_r : vh_t;
        for (int k = lane; k < n * n; k += 64) {
            const int r = k / n, c = k - r * n;
            const d2 v = sh.X[r * ld + c];
            q[k] = quant(v);
            if (vh_out) vh_out[b * n * n + k] = v;
        }
        wsync();
    }
    if (!ok) st |= ACE_ST_BF_NOCONV;
    // ---------------- received-power search (codebook_library.py:67-77)
    // wr_quant[b', j] = j^(-qr[j][b']) (b', j < rx), wt_quant[a, i] = j^(-qt[i][a]) (a, i < tx)
    d2* Hs = sh.A;
    d2* T = sh.X;
    for (int k = lane; k < nh; k += 64) {
        const int r = k / rx, c = k - r * rx;
        Hs[r * ld + c] = Hb[k];
    }
    wsync();
    for (int k = lane; k < nh; k += 64) {  // T[a][j] = sum_b H[a][b] wr[b][j]
        const int a = k / rx, j = k - a * rx;
        d2 acc = make_double2(0.0, 0.0);
        for (int bb = 0; bb < rx; ++bb) acc = cadd(acc, rotk(Hs[a * ld + bb], -sh.qr[j * rx + bb]));
        T[a * ld + j] = acc;
    }
    wsync();
    double best = -__builtin_inf();
    int bidx = 0x7fffffff;
    for (int k = lane; k < nh; k += 64) {  // M[i][j] = sum_a wt[a][i] T[a][j], i-major (i < tx, j < rx)
        const int i = k / rx, j = k - i * rx;
        d2 acc = make_double2(0.0, 0.0);
        for (int a = 0; a < tx; ++a) acc = cadd(acc, rotk(T[a * ld + j], -sh.qt[i * tx + a]));
        const double amp = hypot(acc.x, acc.y);
        const double rss = 10.0 * log10(amp * amp * 1000.0);
        if (bf_better(rss, k, best, bidx)) { best = rss; bidx = k; }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bidx, o, 64);
        if (bf_better(ob, oi, best, bidx)) { best = ob; bidx = oi; }
    }
    const int tx_idx = bidx / rx, rx_idx = bidx - tx_idx * rx;
    // offset [batch][N]: entry k compensates element k of both codes (numpy broadcasting of the reference's
    // `* np.exp(-1j * offset)`, :122-127; tx != rx admits only a constant offset there)
    const bool has_off = offset != nullptr;
    for (int k = lane; k < rx; k += 64)
        wr_code[b * rx + k] = code_of(sh.qr[rx_idx * rx + k], has_off, has_off ? offset[b * N + k] : 0.0);
    for (int k = lane; k < tx; k += 64)
        wt_code[b * tx + k] = code_of(sh.qt[tx_idx * tx + k], has_off, has_off ? offset[b * N + k] : 0.0);
    if (lane == 0) {
        beam_idx[2 * b] = tx_idx;
        beam_idx[2 * b + 1] = rx_idx;
        rss_out[b] = best;
        status[b] = st;
    }
}

size_t bf_lds_bytes(int tx, int rx) {
    const size_t N = std::max(tx, rx);
    return (size_t)(tx != rx ? 3 : 2) * N * (N + 1) * sizeof(d2) + BF_NMAX * sizeof(d2) +
           2 * BF_NMAX * sizeof(double) + (size_t)tx * tx + (size_t)rx * rx;
}

}  // namespace
}  // namespace ace

using namespace ace;

extern "C" int ace_svd_beamformer_batch(int batch, int tx, int rx, const double* H, const double* offset,
                                        uint8_t* wr_code, uint8_t* wt_code, int32_t* beam_idx, double* rss,
                                        uint32_t* status, double* vh_r, double* vh_t, void* stream) {
    g_err.clear();
    if (batch < 0) return fail(ACE_ERR_ARG, "svd_beamformer: batch %d < 0", batch);
    if (tx < 1 || tx > BF_NMAX || rx < 1 || rx > BF_NMAX)
        return fail(ACE_ERR_UNSUPPORTED, "svd_beamformer: %d x %d antennas outside 1..%d", tx, rx, BF_NMAX);
    if (batch == 0) return ACE_OK;
    if (!H || !wr_code || !wt_code || !beam_idx || !rss || !status)
        return fail(ACE_ERR_ARG, "svd_beamformer: null output/input pointer");
    const size_t lds = bf_lds_bytes(tx, rx);
    hipLaunchKernelGGL(tx == rx ? beamformer_kernel<false> : beamformer_kernel<true>, dim3(batch), dim3(64), lds,
                       (hipStream_t)stream, tx, rx, (const d2*)H, offset,
                       wr_code, wt_code, beam_idx, rss, status, (d2*)vh_r, (d2*)vh_t);
    ACE_HIP(hipGetLastError());
    return ACE_OK;
}

extern "C" int ace_svd_beamformer_host(int batch, int tx, int rx, const double* H, const double* offset,
                                       uint8_t* wr_code, uint8_t* wt_code, int32_t* beam_idx, double* rss,
                                       uint32_t* status, double* vh_r, double* vh_t) {
    g_err.clear();
    if (batch < 0 || tx < 1 || tx > BF_NMAX || rx < 1 || rx > BF_NMAX)
        return ace_svd_beamformer_batch(batch, tx, rx, H, offset, wr_code, wt_code, beam_idx, rss, status, vh_r,
                                        vh_t, nullptr);
    if (batch == 0) return ACE_OK;
    const size_t B = batch, N = std::max(tx, rx), nH = 16 * B * tx * rx, nvr = 16 * B * rx * rx,
                 nvt = 16 * B * tx * tx, noff = 8 * B * N, ncr = B * rx, nct = B * tx;
    std::vector<void*> bufs;
    auto cleanup = [&]() {
        for (void* q : bufs) (void)hipFree(q);
        bufs.clear();
    };
    auto dalloc = [&](size_t bytes, void** q) -> hipError_t {
        hipError_t e = hipMalloc(q, bytes);
        if (e == hipSuccess) bufs.push_back(*q);
        return e;
    };
    void *dH, *doff = nullptr, *dwr, *dwt, *didx, *drss, *dst, *dvr = nullptr, *dvt = nullptr;
    hipError_t e;
    if ((e = dalloc(nH, &dH)) || (offset && (e = dalloc(noff, &doff))) || (e = dalloc(ncr, &dwr)) ||
        (e = dalloc(nct, &dwt)) || (e = dalloc(8 * B, &didx)) || (e = dalloc(8 * B, &drss)) ||
        (e = dalloc(4 * B, &dst)) || (vh_r && (e = dalloc(nvr, &dvr))) || (vh_t && (e = dalloc(nvt, &dvt)))) {
        cleanup();
        return fail(ACE_ERR_HIP, "hipMalloc: %s", hipGetErrorString(e));
    }
    if ((e = hipMemcpy(dH, H, nH, hipMemcpyHostToDevice)) ||
        (offset && (e = hipMemcpy(doff, offset, noff, hipMemcpyHostToDevice)))) {
        cleanup();
        return fail(ACE_ERR_HIP, "hipMemcpy: %s", hipGetErrorString(e));
    }
    int rc = ace_svd_beamformer_batch(batch, tx, rx, (const double*)dH, (const double*)doff, (uint8_t*)dwr,
                                      (uint8_t*)dwt, (int32_t*)didx, (double*)drss, (uint32_t*)dst, (double*)dvr,
                                      (double*)dvt, nullptr);
    if (rc == ACE_OK) {
        if ((e = hipDeviceSynchronize()) || (e = hipMemcpy(wr_code, dwr, ncr, hipMemcpyDeviceToHost)) ||
            (e = hipMemcpy(wt_code, dwt, nct, hipMemcpyDeviceToHost)) ||
            (e = hipMemcpy(beam_idx, didx, 8 * B, hipMemcpyDeviceToHost)) ||
            (e = hipMemcpy(rss, drss, 8 * B, hipMemcpyDeviceToHost)) ||
            (e = hipMemcpy(status, dst, 4 * B, hipMemcpyDeviceToHost)) ||
            (vh_r && (e = hipMemcpy(vh_r, dvr, nvr, hipMemcpyDeviceToHost))) ||
            (vh_t && (e = hipMemcpy(vh_t, dvt, nvt, hipMemcpyDeviceToHost))))
            rc = fail(ACE_ERR_HIP, "svd_beamformer: %s", hipGetErrorString(e));
    }
    const std::string keep = g_err;
    cleanup();
    g_err = keep;
    return rc;
}
