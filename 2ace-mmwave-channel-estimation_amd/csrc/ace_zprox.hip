// Per-realisation kernels of the ADMM iteration (one work-group per realisation):
//   pre   : V = Z - N/mu, S = Y - M/mu                       (operands of ArgMinX)
//   ystep : AX = S - g, ArgMinY, M update, m-space reductions (inferLowRankV4_multi.m:329,:336-337,:345)
//   zstep : ArgMinZ (A2only spectral tail rescale via a Hermitian Jacobi eigensolver
//           of the tx x tx matrix E E^H in LDS; nuclear: norm shrink), N update,
//           residuals, convergence test, best-objective tracking, mu update
//           (:333, :340-341, :344-382)
//
// ArgMinX runs in Woodbury form.  With G = (I + A A^H)^{-1} and K = A A^H:
//   inv(A^H A + I) (A^H s + v) = v + A^H G (s - A v),     A X = s - G (s - A v),
//   ||A^H d||^2 = d^H K d.
// This is algebraically identical to the reference's X = U (A'(Y-M/mu) + Z-N/mu)
// (:325, ArgMinX :404) and to its A'*Y residual terms (:330, :365, :369); it
// replaces the n x n apply by m x m ones.
#include "ace_common.hpp"

namespace ace {

namespace {
constexpr int TXMAX = 32;
constexpr int HS = TXMAX + 1;  // LDS row stride (complex) for 32x32 tiles
constexpr int MAX_SWEEPS = 40;

// Circle-method pairing: step s of n-1, pair k of n/2 -> (p, q) with p < q.
__device__ __forceinline__ void rr_pair(int n, int s, int k, int& p, int& q) {
    int a, b;
    if (k == 0) {
        a = n - 1;
        b = s;
    } else {
        a = (s + k) % (n - 1);
        b = (s - k + (n - 1)) % (n - 1);
    }
    p = a < b ? a : b;
    q = a < b ? b : a;
}

template <int VARIANT, bool INIT>
__global__ __launch_bounds__(256) void zstep_kernel(ZArgs a) {
    const int b = blockIdx.x;
    const int t = threadIdx.x, nt = blockDim.x;
    const int n = a.n, m = a.m, tx = a.tx, rx = a.rx;
    RealState* st = a.st + b;
    __shared__ double red[16 * 8];
    __shared__ int flag_rot, flag_improved, flag_any;
    if (!INIT && st->done) return;
    const double mu = INIT ? 1.0 : st->mu;
    const double imu = 1.0 / mu;
    const d2* X = reinterpret_cast<const d2*>(a.X) + (long long)b * n;
    d2* N = reinterpret_cast<d2*>(a.N) + (long long)b * n;
    d2* Z = reinterpret_cast<d2*>(a.Z) + (long long)b * n;

    // accumulators: nX2, nZ2, nJN2, dZ2
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    auto emit = [&](int k, d2 znew) {  // per-element update + reductions
        const d2 x = X[k];
        if (!INIT) {
            const d2 zo = Z[k];
            const d2 d = csub(x, znew);
            N[k] = cadd(N[k], cscale(d, mu));
            acc[0] += cabs2(x);
            acc[1] += cabs2(znew);
            acc[2] += cabs2(d);
            acc[3] += cabs2(csub(znew, zo));
        }
        Z[k] = znew;
    };
    // E = reshape(X + N/mu, tx, []) : E[i][j] = z[i + tx*j]   (:424-426)
    auto evalE = [&](int k) -> d2 { return cadd(X[k], cscale(N[k], imu)); };

    if constexpr (VARIANT == ACE_VARIANT_NUCLEAR) {
        // inferLowRank_Nuclear.m:411-419 at r = 1: Z = z * max(0, ||z|| - 1/mu) / ||z||
        double s[1] = {0.0};
        for (int k = t; k < n; k += nt) s[0] += cabs2(evalE(k));
        block_sum<1>(s, red);
        const double nz = sqrt(s[0]);
        const double f = nz > 0.0 ? fmax(0.0, nz - imu) / nz : 0.0;
        for (int k = t; k < n; k += nt) emit(k, cscale(evalE(k), f));
    } else {
        __shared__ d2 Hs[TXMAX * HS];
        __shared__ d2 Qs[TXMAX * HS];
        __shared__ d2 Ts[TXMAX * HS];
        __shared__ double rc[TXMAX / 2], rs[TXMAX / 2];
        __shared__ d2 re[TXMAX / 2];
        __shared__ int rp[TXMAX / 2], rq[TXMAX / 2];
        __shared__ double wv[TXMAX], scl[TXMAX], rs2[TXMAX];
        __shared__ int ord[TXMAX], ascp[TXMAX];
        // E into Ts
        for (int e = t; e < tx * rx; e += nt) {
            const int i = e % tx, j = e / tx;
            Ts[i * HS + j] = evalE(e);
        }
        __syncthreads();
        // H = E E^H  (:428)
        for (int e = t; e < tx * tx; e += nt) {
            const int i = e / tx, i2 = e % tx;
            d2 s = make_double2(0.0, 0.0);
            for (int j = 0; j < rx; ++j) {
                const d2 u = Ts[i * HS + j], v = Ts[i2 * HS + j];
                s.x += u.x * v.x + u.y * v.y;  // u * conj(v)
                s.y += u.y * v.x - u.x * v.y;
            }
            if (i == i2) s.y = 0.0;
            Hs[i * HS + i2] = s;
        }
        const bool warm = (!INIT) && a.warm && a.Q;
        d2* Qg = a.Q ? reinterpret_cast<d2*>(a.Q) + (long long)b * tx * tx : nullptr;
        if (warm) {
            for (int e = t; e < tx * tx; e += nt) Qs[(e / tx) * HS + (e % tx)] = Qg[e];
            __syncthreads();
            // Ts = H Q ; H = Q^H Ts
            for (int e = t; e < tx * tx; e += nt) {
                const int i = e / tx, c = e % tx;
                d2 s = make_double2(0.0, 0.0);
                for (int k = 0; k < tx; ++k) s = cadd(s, cmul(Hs[i * HS + k], Qs[k * HS + c]));
                Ts[i * HS + c] = s;
            }
            __syncthreads();
            for (int e = t; e < tx * tx; e += nt) {
                const int r = e / tx, c = e % tx;
                d2 s = make_double2(0.0, 0.0);
                for (int k = 0; k < tx; ++k) s = cadd(s, cmulc(Qs[k * HS + r], Ts[k * HS + c]));
                Hs[r * HS + c] = s;
            }
            __syncthreads();
            // re-Hermitise: H = (H + H^H)/2 (upper from lower)
            for (int e = t; e < tx * tx; e += nt) {
                const int r = e / tx, c = e % tx;
                if (r < c) {
                    const d2 u = Hs[r * HS + c], l = Hs[c * HS + r];
                    const d2 h = make_double2(0.5 * (u.x + l.x), 0.5 * (u.y - l.y));
                    Hs[r * HS + c] = h;
                    Hs[c * HS + r] = make_double2(h.x, -h.y);
                } else if (r == c) {
                    Hs[r * HS + c].y = 0.0;
                }
            }
        } else {
            for (int e = t; e < tx * tx; e += nt) {
                const int i = e / tx, c = e % tx;
                Qs[i * HS + c] = make_double2(i == c ? 1.0 : 0.0, 0.0);
            }
        }
        __syncthreads();
        double tr = 0.0;
        for (int k = 0; k < tx; ++k) tr += fabs(Hs[k * HS + k].x);
        const double abs_tol = 1e-18 * tr;
        const int P = tx / 2;
        int sweeps = 0;
        // Parallel cyclic Jacobi: every step applies P disjoint rotations as one
        // block-diagonal unitary J: H <- J^H H J, Q <- Q J.
        for (; sweeps < MAX_SWEEPS; ++sweeps) {
            if (t == 0) flag_rot = 0;
            __syncthreads();
            for (int s = 0; s < tx - 1; ++s) {
                if (t < P) {
                    int p, q;
                    rr_pair(tx, s, t, p, q);
                    const double ap = Hs[p * HS + p].x, aq = Hs[q * HS + q].x;
                    const d2 c = Hs[p * HS + q];
                    const double ac = sqrt(cabs2(c));
                    double cs = 1.0, sn = 0.0;
                    d2 ep = make_double2(1.0, 0.0);
                    if (ac > abs_tol && ac * ac > 1e-32 * fabs(ap * aq) && ac > 1e-300) {
                        ep = make_double2(c.x / ac, c.y / ac);
                        const double zeta = (aq - ap) / (2.0 * ac);
                        const double tt = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                        cs = 1.0 / sqrt(1.0 + tt * tt);
                        sn = tt * cs;
                        flag_rot = 1;
                    }
                    rc[t] = cs;
                    rs[t] = sn;
                    re[t] = ep;
                    rp[t] = p;
                    rq[t] = q;
                }
                __syncthreads();
                // H blocks (ka, kb): H'[a,b] = Ja^H H[a,b] Jb, J = [[cs, sn], [-sn e*, cs e*]]
                for (int e = t; e < P * P; e += nt) {
                    const int ka = e / P, kb = e % P;
                    const int pa = rp[ka], qa = rq[ka], pb = rp[kb], qb = rq[kb];
                    const double ca = rc[ka], sa = rs[ka], cb = rc[kb], sb = rs[kb];
                    const d2 ea = re[ka], eb = re[kb];
                    const d2 h00 = Hs[pa * HS + pb], h01 = Hs[pa * HS + qb];
                    const d2 h10 = Hs[qa * HS + pb], h11 = Hs[qa * HS + qb];
                    const d2 ebc = make_double2(eb.x, -eb.y);
                    // T = H Jb
                    const d2 t01 = cmul(h01, ebc), t11 = cmul(h11, ebc);
                    const d2 T00 = csub(cscale(h00, cb), cscale(t01, sb));
                    const d2 T01 = cadd(cscale(h00, sb), cscale(t01, cb));
                    const d2 T10 = csub(cscale(h10, cb), cscale(t11, sb));
                    const d2 T11 = cadd(cscale(h10, sb), cscale(t11, cb));
                    // H' = Ja^H T : row0 = ca*T0 - sa*ea*T1, row1 = sa*T0 + ca*ea*T1
                    const d2 u10 = cmul(ea, T10), u11 = cmul(ea, T11);
                    Hs[pa * HS + pb] = csub(cscale(T00, ca), cscale(u10, sa));
                    Hs[pa * HS + qb] = csub(cscale(T01, ca), cscale(u11, sa));
                    Hs[qa * HS + pb] = cadd(cscale(T00, sa), cscale(u10, ca));
                    Hs[qa * HS + qb] = cadd(cscale(T01, sa), cscale(u11, ca));
                }
                for (int e = t; e < tx * P; e += nt) {
                    const int i = e / P, kb = e % P;
                    const int pb = rp[kb], qb = rq[kb];
                    const double cb = rc[kb], sb = rs[kb];
                    const d2 eb = re[kb];
                    const d2 qp = Qs[i * HS + pb];
                    const d2 qq = cmul(Qs[i * HS + qb], make_double2(eb.x, -eb.y));
                    Qs[i * HS + pb] = csub(cscale(qp, cb), cscale(qq, sb));
                    Qs[i * HS + qb] = cadd(cscale(qp, sb), cscale(qq, cb));
                }
                __syncthreads();
            }
            if (!flag_rot) break;
            __syncthreads();
        }
        if (sweeps >= MAX_SWEEPS && t == 0) atomicOr(&st->status, (int)ACE_ST_EIG_NOCONV);
        // eigenvalues; MATLAB order emulation: ascending (LAPACK) then stable descending (:429-430)
        if (t < tx) wv[t] = Hs[t * HS + t].x;
        __syncthreads();
        if (t < tx) {  // position in LAPACK's ascending order
            const double wk = wv[t];
            int asc = 0;
            for (int j = 0; j < tx; ++j) asc += (wv[j] < wk) || (wv[j] == wk && j < t);
            ascp[t] = asc;
        }
        __syncthreads();
        if (t < tx) {  // stable descending rank of max(0, w)
            const double sk = fmax(0.0, wv[t]);
            const int asc = ascp[t];
            int rank = 0;
            for (int j = 0; j < tx; ++j) {
                const double sj = fmax(0.0, wv[j]);
                rank += (sj > sk) || (sj == sk && ascp[j] < asc);
            }
            ord[rank] = t;  // ord[sorted position] = eigen index
            scl[t] = 1.0;
        }
        __syncthreads();
        if (t == 0) {  // rank-profile tail rescaling (:469-480), sequential sums
            double* s2 = rs2;
            for (int k = 0; k < tx; ++k) s2[k] = fmax(0.0, wv[ord[k]]);
            for (int pi = 0; pi < a.np; ++pi) {
                const int r = a.rl[pi];
                const double f = a.fl[pi];
                double vr = 0.0, v = 0.0;
                for (int k = 0; k < r; ++k) vr += s2[k];
                for (int k = 0; k < tx; ++k) v += s2[k];
                if (vr < v * f) {
                    const double sc = fmin(1.0, vr / (v - vr) * (1.0 / f - 1.0));
                    for (int k = r; k < tx; ++k) {
                        s2[k] *= sc;
                        scl[ord[k]] *= sc;
                    }
                }
            }
            int any = 0;
            for (int k = 0; k < tx; ++k) any |= scl[k] < 1.0;
            flag_any = any;
        }
        __syncthreads();
        if (flag_any) {
            // Z = U diag(sqrt(scl)) U^H E  (:482-484); E restaged into Hs
            for (int e = t; e < tx * rx; e += nt) {
                const int i = e % tx, j = e / tx;
                Hs[i * HS + j] = evalE(e);
            }
            __syncthreads();
            for (int e = t; e < tx * rx; e += nt) {
                const int c = e / rx, j = e % rx;
                d2 s = make_double2(0.0, 0.0);
                for (int i = 0; i < tx; ++i) s = cadd(s, cmulc(Qs[i * HS + c], Hs[i * HS + j]));
                Ts[c * HS + j] = cscale(s, sqrt(scl[c]));
            }
            __syncthreads();
            for (int e = t; e < tx * rx; e += nt) {
                const int i = e % tx, j = e / tx;
                d2 s = make_double2(0.0, 0.0);
                for (int c = 0; c < tx; ++c) s = cadd(s, cmul(Qs[i * HS + c], Ts[c * HS + j]));
                emit(e, s);
            }
        } else {
            for (int k = t; k < n; k += nt) emit(k, evalE(k));
        }
        if (a.Q) {
            for (int e = t; e < tx * tx; e += nt) Qg[e] = Qs[(e / tx) * HS + (e % tx)];
        }
    }
    if (INIT) return;

    // m-space dual terms: ||A^H (Y - Y0)||^2 = dY^H (K Y - K Y0),  ||A^H Y||^2 = Y^H K Y
    double v6[6] = {acc[0], acc[1], acc[2], acc[3], 0.0, 0.0};
    {
        const d2* Yn = reinterpret_cast<const d2*>(a.Ynew) + (long long)b * m;
        const d2* Yo = reinterpret_cast<const d2*>(a.Yold) + (long long)b * m;
        const d2* Kn = reinterpret_cast<const d2*>(a.KYnew) + (long long)b * m;
        const d2* Ko = reinterpret_cast<const d2*>(a.KYold) + (long long)b * m;
        for (int i = t; i < m; i += nt) {
            const d2 yn = Yn[i], kn = Kn[i];
            const d2 dy = csub(yn, Yo[i]), dk = csub(kn, Ko[i]);
            v6[4] += dy.x * dk.x + dy.y * dk.y;
            v6[5] += yn.x * kn.x + yn.y * kn.y;
        }
    }
    block_sum<6>(v6, red);
    if (t == 0) {
        const double nX = sqrt(v6[0]), nZ = sqrt(v6[1]), jn2 = v6[2], dZ2 = v6[3];
        const double dAtY2 = fmax(0.0, v6[4]), nAtY2 = fmax(0.0, v6[5]);
        const double obj = sqrt(st->obj2);
        const double nAX = sqrt(st->nAX2), nY = sqrt(st->nY2);
        const double r = 1.0;  // columns per realisation
        int improved = 0;
        if (obj < st->opt_obj) {  // :344-351
            st->opt_obj = obj;
            improved = 1;
        }
        flag_improved = improved;
        const double res_prim = sqrt(st->nJM2 + jn2);  // :364-366
        const double res_dual = mu * sqrt(dAtY2 + dZ2);
        const double res_comb = sqrt(res_prim * res_prim + st->dY2 + dZ2);
        const double mx1 = fmax(nAX, nY), mx2 = fmax(nX, nZ);  // :368-370
        const double t_prim = a.tol_abs * sqrt((double)(m + n) * r) + a.tol_rel * sqrt(mx1 * mx1 + mx2 * mx2);
        const double t_dual = a.tol_abs * sqrt((double)n * r * 2) + a.tol_rel * sqrt(nAtY2 + nZ * nZ);
        const double t_comb = a.tol_abs * sqrt((double)(m + n) * r * 2) +
                              a.tol_rel * sqrt(mx1 * mx1 + mx2 * mx2 + nY * nY + nZ * nZ);
        st->iters = a.it;
        const bool conv = (res_prim < t_prim && res_dual < t_dual) || (res_comb < t_comb);  // :372
        bool stop = false;
        if (conv) {
            st->status |= ACE_ST_CONVERGED;
            if (!a.fixed_iters) stop = true;
        }
        if (stop) {
            st->done = 1;
            atomicAdd(a.done_count, 1);
        } else {
            if (res_comb > st->last_res * 0.9) st->mu = mu * a.rho;  // :379-381
            st->last_res = res_comb;
        }
    }
    __syncthreads();
    if (flag_improved) {
        d2* oX = reinterpret_cast<d2*>(a.optX) + (long long)b * n;
        d2* oY = reinterpret_cast<d2*>(a.optY) + (long long)b * m;
        const d2* Yn = reinterpret_cast<const d2*>(a.Ynew) + (long long)b * m;
        for (int k = t; k < n; k += nt) oX[k] = X[k];
        for (int i = t; i < m; i += nt) oY[i] = Yn[i];
    }
}

// V = Z - N/mu (n), S = Y - M/mu (m)
__global__ __launch_bounds__(256) void pre_kernel(int n, int m, const double* Zp, const double* Np, const double* Yp,
                                                  const double* Mp, double* Vp, double* Sp, const RealState* st) {
    const int b = blockIdx.x;
    if (st[b].done) return;
    const double imu = 1.0 / st[b].mu;
    const d2* Z = reinterpret_cast<const d2*>(Zp) + (long long)b * n;
    const d2* N = reinterpret_cast<const d2*>(Np) + (long long)b * n;
    d2* V = reinterpret_cast<d2*>(Vp) + (long long)b * n;
    for (int k = threadIdx.x; k < n; k += blockDim.x) V[k] = csub(Z[k], cscale(N[k], imu));
    const d2* Y = reinterpret_cast<const d2*>(Yp) + (long long)b * m;
    const d2* M = reinterpret_cast<const d2*>(Mp) + (long long)b * m;
    d2* S = reinterpret_cast<d2*>(Sp) + (long long)b * m;
    for (int i = threadIdx.x; i < m; i += blockDim.x) S[i] = csub(Y[i], cscale(M[i], imu));
}

// Y-step (r = 1): AX = S - g, C = AX + M/mu, Y = C (B/|C| + mu)/(1 + mu), M += mu (AX - Y)
__global__ __launch_bounds__(256) void ystep_kernel(int m, const double* Sp, const double* gp, double* Mp,
                                                    const double* Bp, const double* Yold, double* Ynew,
                                                    RealState* st) {
    const int b = blockIdx.x;
    __shared__ double red[16 * 5];
    if (st[b].done) return;
    const double mu = st[b].mu, imu = 1.0 / mu;
    const d2* S = reinterpret_cast<const d2*>(Sp) + (long long)b * m;
    const d2* g = reinterpret_cast<const d2*>(gp) + (long long)b * m;
    d2* M = reinterpret_cast<d2*>(Mp) + (long long)b * m;
    const double* B = Bp + (long long)b * m;
    const d2* Yo = reinterpret_cast<const d2*>(Yold) + (long long)b * m;
    d2* Yn = reinterpret_cast<d2*>(Ynew) + (long long)b * m;
    double v[5] = {0, 0, 0, 0, 0};  // obj2, nAX2, nY2, nJM2, dY2
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const d2 ax = csub(S[i], g[i]);
        const d2 mi = M[i];
        d2 c = cadd(ax, cscale(mi, imu));
        double d = sqrt(cabs2(c));
        if (d == 0.0) {  // ArgMinY zero guard (:516-520 / :524-528)
            c = make_double2(1.0, 0.0);
            d = 1.0;
        }
        const double f = (B[i] / d + mu) / (1.0 + mu);
        const d2 y = cscale(c, f);
        const d2 j = csub(ax, y);
        M[i] = cadd(mi, cscale(j, mu));
        Yn[i] = y;
        const double aax = sqrt(cabs2(ax)) - B[i];
        v[0] += aax * aax;
        v[1] += cabs2(ax);
        v[2] += cabs2(y);
        v[3] += cabs2(j);
        v[4] += cabs2(csub(y, Yo[i]));
    }
    block_sum<5>(v, red);
    if (threadIdx.x == 0) {
        st[b].obj2 = v[0];
        st[b].nAX2 = v[1];
        st[b].nY2 = v[2];
        st[b].nJM2 = v[3];
        st[b].dY2 = v[4];
    }
}

// Initialisation (InferADMM :296-308): P0 = A X0 given; scale X0, AX; Y = normalize_rows(AX,B); M = N = 0.
__global__ __launch_bounds__(256) void init_kernel(int n, int m, const double* X0p, const double* P0p,
                                                   const double* Bp, double* Xp, double* Yp, double* Mp,
                                                   double* Np, RealState* st, double mu0) {
    const int b = blockIdx.x;
    __shared__ double red[16 * 2];
    const d2* X0 = reinterpret_cast<const d2*>(X0p) + (long long)b * n;
    const d2* P0 = reinterpret_cast<const d2*>(P0p) + (long long)b * m;
    const double* B = Bp + (long long)b * m;
    double v[2] = {0.0, 0.0};
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        v[0] += B[i] * B[i];
        v[1] += cabs2(P0[i]);
    }
    block_sum<2>(v, red);
    const double nB = sqrt(v[0]), s = nB / sqrt(v[1]);  // :301 X * (norm(B)/norm(AX,'fro'))
    d2* X = reinterpret_cast<d2*>(Xp) + (long long)b * n;
    d2* N = reinterpret_cast<d2*>(Np) + (long long)b * n;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        X[k] = cscale(X0[k], s);
        N[k] = make_double2(0.0, 0.0);
    }
    d2* Y = reinterpret_cast<d2*>(Yp) + (long long)b * m;
    d2* M = reinterpret_cast<d2*>(Mp) + (long long)b * m;
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        d2 ax = cscale(P0[i], s);
        double d = sqrt(cabs2(ax));
        if (d == 0.0) {
            ax = make_double2(1.0, 0.0);
            d = 1.0;
        }
        Y[i] = cscale(ax, B[i] / d);  // normalize_rows (:538-559)
        M[i] = make_double2(0.0, 0.0);
    }
    if (threadIdx.x == 0) {
        RealState r = {};
        r.mu = mu0;
        r.last_res = INFINITY;
        r.opt_obj = INFINITY;
        r.nB = nB;
        st[b] = r;
    }
}

__global__ __launch_bounds__(256) void finalize_kernel(int n, int m, const double* optX, const double* optY,
                                                       const double* Xcur, const double* Ycur, double* Xo,
                                                       double* Yo, int32_t* iters, uint32_t* status, double* muo,
                                                       RealState* st) {
    const int b = blockIdx.x;
    const bool have = st[b].opt_obj < INFINITY;
    const d2* sx = reinterpret_cast<const d2*>(have ? optX : Xcur) + (long long)b * n;
    const d2* sy = reinterpret_cast<const d2*>(have ? optY : Ycur) + (long long)b * m;
    d2* dx = reinterpret_cast<d2*>(Xo) + (long long)b * n;
    d2* dy = reinterpret_cast<d2*>(Yo) + (long long)b * m;
    for (int k = threadIdx.x; k < n; k += blockDim.x) dx[k] = sx[k];
    for (int i = threadIdx.x; i < m; i += blockDim.x) dy[i] = sy[i];
    if (threadIdx.x == 0) {
        if (iters) iters[b] = st[b].iters;
        if (status) status[b] = (uint32_t)st[b].status | (have ? 0u : ACE_ST_NO_OPT);
        if (muo) muo[b] = st[b].mu;
    }
}

// A^H (conjugate transpose), 32x32 LDS tiles: AH[k][i] = conj(A[i][k])
__global__ __launch_bounds__(256) void conj_transpose_kernel(int rows, int cols, const double* Ap, double* AHp) {
    __shared__ d2 tile[32][33];
    const d2* A = reinterpret_cast<const d2*>(Ap);
    d2* AH = reinterpret_cast<d2*>(AHp);
    const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
    const int tx_ = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int y = ty; y < 32; y += 8) {
        const int r = r0 + y, c = c0 + tx_;
        if (r < rows && c < cols) tile[y][tx_] = A[(long long)r * cols + c];
    }
    __syncthreads();
    for (int y = ty; y < 32; y += 8) {
        const int c = c0 + y, r = r0 + tx_;
        if (r < rows && c < cols) {
            const d2 v = tile[tx_][y];
            AH[(long long)c * rows + r] = make_double2(v.x, -v.y);
        }
    }
}
}  // namespace

void launch_zstep(int variant, bool init, const ZArgs& a, int batch, hipStream_t st) {
    if (variant == ACE_VARIANT_NUCLEAR) {
        if (init) hipLaunchKernelGGL((zstep_kernel<ACE_VARIANT_NUCLEAR, true>), dim3(batch), dim3(256), 0, st, a);
        else hipLaunchKernelGGL((zstep_kernel<ACE_VARIANT_NUCLEAR, false>), dim3(batch), dim3(256), 0, st, a);
    } else {
        if (init) hipLaunchKernelGGL((zstep_kernel<ACE_VARIANT_A2ONLY, true>), dim3(batch), dim3(256), 0, st, a);
        else hipLaunchKernelGGL((zstep_kernel<ACE_VARIANT_A2ONLY, false>), dim3(batch), dim3(256), 0, st, a);
    }
}
void launch_pre(int n, int m, int batch, const double* Z, const double* N, const double* Y, const double* M, double* V,
                double* S, const RealState* rs, hipStream_t st) {
    hipLaunchKernelGGL(pre_kernel, dim3(batch), dim3(256), 0, st, n, m, Z, N, Y, M, V, S, rs);
}
void launch_ystep(int m, int batch, const double* S, const double* g, double* M, const double* B, const double* Yold,
                  double* Ynew, RealState* rs, hipStream_t st) {
    hipLaunchKernelGGL(ystep_kernel, dim3(batch), dim3(256), 0, st, m, S, g, M, B, Yold, Ynew, rs);
}
void launch_init(int n, int m, int batch, const double* X0, const double* P0, const double* B, double* X, double* Y,
                 double* M, double* N, RealState* rs, double mu0, hipStream_t st) {
    hipLaunchKernelGGL(init_kernel, dim3(batch), dim3(256), 0, st, n, m, X0, P0, B, X, Y, M, N, rs, mu0);
}
void launch_finalize(int n, int m, int batch, const double* optX, const double* optY, const double* Xc,
                     const double* Yc, double* Xo, double* Yo, int32_t* iters, uint32_t* status, double* mu,
                     RealState* rs, hipStream_t st) {
    hipLaunchKernelGGL(finalize_kernel, dim3(batch), dim3(256), 0, st, n, m, optX, optY, Xc, Yc, Xo, Yo, iters, status,
                       mu, rs);
}
void launch_conj_transpose(int rows, int cols, const double* A, double* AH, hipStream_t st) {
    dim3 grid((cols + 31) / 32, (rows + 31) / 32);
    hipLaunchKernelGGL(conj_transpose_kernel, grid, dim3(256), 0, st, rows, cols, A, AH);
}

}  // namespace ace
