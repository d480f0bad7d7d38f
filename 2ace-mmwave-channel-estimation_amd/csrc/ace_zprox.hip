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
#include "ace_zcommon.hpp"

namespace ace {

namespace {
constexpr int TXMAX = 32;
constexpr int HS = TXMAX + 1;  // LDS row stride (complex) for 32x32 tiles
constexpr int MAX_SWEEPS = 40;

// 32x32 complex product from LDS tiles (row stride HS) on the f64 matrix cores:
// C = opA(A) * opB(B), op = identity or conjugate transpose.  Wave w computes the
// 16x16 block rows [16*(w>>1), +16) x cols [16*(w&1), +16); real and imaginary
// parts accumulate in separate 16x16 f64 tiles (4 real MFMAs per complex k-step).
template <bool CTA, bool CTB>
__device__ __forceinline__ void mm32(const d2* A, const d2* B, d4v& cr, d4v& ci, int lane, int w) {
    const int i0 = 16 * (w >> 1), j0 = 16 * (w & 1);
    cr = d4v{0.0, 0.0, 0.0, 0.0};
    ci = d4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k0 = 0; k0 < 32; k0 += 4) {
        const int kk = k0 + (lane >> 4);
        d2 av = CTA ? A[kk * HS + i0 + (lane & 15)] : A[(i0 + (lane & 15)) * HS + kk];
        d2 bv = CTB ? B[(j0 + (lane & 15)) * HS + kk] : B[kk * HS + j0 + (lane & 15)];
        if (CTA) av.y = -av.y;
        if (CTB) bv.y = -bv.y;
        cr = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.x, cr, 0, 0, 0);
        cr = __builtin_amdgcn_mfma_f64_16x16x4f64(-av.y, bv.y, cr, 0, 0, 0);
        ci = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.y, ci, 0, 0, 0);
        ci = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bv.x, ci, 0, 0, 0);
    }
}
// store an mm32 result: lane l, reg r -> row i0 + (l>>4) + 4r, col j0 + (l&15)
__device__ __forceinline__ void store32(d2* C, const d4v& cr, const d4v& ci, int lane, int w) {
    const int i0 = 16 * (w >> 1), j0 = 16 * (w & 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) C[(i0 + (lane >> 4) + 4 * r) * HS + j0 + (lane & 15)] = make_double2(cr[r], ci[r]);
}

template <int VARIANT, bool INIT>
__global__ __launch_bounds__(256) void zstep_kernel(ZArgs a) {
    const int b = blockIdx.x;
    const int t = threadIdx.x, nt = blockDim.x;
    const int n = a.n, m = a.m, tx = a.tx, rx = a.rx;
    RealState* st = a.st + b;
    __shared__ double red[16 * 8];
    __shared__ int flag_improved, flag_any;
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
        // ---- A2only ArgMinZ (inferLowRankV4_multi.m:423-485) ------------------------
        // Two 32x32 complex LDS tiles (E/H/T in L0, eigenvectors Q in L1), zero-padded
        // to 32 for tx, rx < 32.  The five 32x32 complex products run on the f64
        // matrix cores (mm32).  The Hermitian eigensolver is a parallel cyclic Jacobi
        // with one barrier per step: every thread derives the two rotations it needs
        // from a double-buffered "rotation input" array (diagonal + the next step's
        // pair entries), written by the threads that produce those entries.
        __shared__ d2 L0[TXMAX * HS];
#ifdef ACE_DEBUG_SWEEPS
        const unsigned long long dbg_t0 = __builtin_amdgcn_s_memrealtime();
        unsigned long long dbg_t1 = 0, dbg_t2 = 0;
#endif
        __shared__ d2 L1[TXMAX * HS];
        __shared__ int flags[MAX_SWEEPS + 1];
        __shared__ double wv[TXMAX], scl[TXMAX], rs2[TXMAX];
        __shared__ int ord[TXMAX], ascp[TXMAX];
        const int lane = t & 63, w = t >> 6;
        if (t <= MAX_SWEEPS) flags[t] = 0;
        // E = reshape(X + N/mu, tx, []) into L0 (zero padded)
        for (int e = t; e < TXMAX * TXMAX; e += nt) {
            const int i = e & 31, j = e >> 5;
            L0[i * HS + j] = (i < tx && j < rx) ? evalE(i + tx * j) : make_double2(0.0, 0.0);
        }
        __syncthreads();
        d4v cr, ci;
        mm32<false, true>(L0, L0, cr, ci, lane, w);      // H = E E^H  (:428)
        __syncthreads();
        store32(L0, cr, ci, lane, w);
        const bool warm = (!INIT) && a.warm && a.Q;
        d2* Qg = a.Q ? reinterpret_cast<d2*>(a.Q) + (long long)b * tx * tx : nullptr;
        for (int e = t; e < TXMAX * TXMAX; e += nt) {
            const int i = e >> 5, c = e & 31;
            d2 q = make_double2(i == c ? 1.0 : 0.0, 0.0);
            if (warm && i < tx && c < tx) q = Qg[i * tx + c];
            L1[i * HS + c] = q;
        }
        __syncthreads();
        if (warm) {  // H <- Q^H H Q: nearly diagonal when Q is last iteration's eigenbasis
            mm32<false, false>(L0, L1, cr, ci, lane, w);  // T = H Q
            __syncthreads();
            store32(L0, cr, ci, lane, w);
            __syncthreads();
            mm32<true, false>(L1, L0, cr, ci, lane, w);   // Q^H T
            __syncthreads();
            store32(L0, cr, ci, lane, w);
            __syncthreads();
            for (int e = t; e < TXMAX * TXMAX; e += nt) {  // exact Hermitian symmetry
                const int r = e >> 5, c = e & 31;
                if (r < c) {
                    const d2 u = L0[r * HS + c], l = L0[c * HS + r];
                    const d2 h = make_double2(0.5 * (u.x + l.x), 0.5 * (u.y - l.y));
                    L0[r * HS + c] = h;
                    L0[c * HS + r] = make_double2(h.x, -h.y);
                } else if (r == c) {
                    L0[r * HS + c].y = 0.0;
                }
            }
            __syncthreads();
        }
        double tr = 0.0;
        for (int k = 0; k < tx; ++k) tr += fabs(L0[k * HS + k].x);
        const double abs_tol = 1e-18 * tr;
        const int P = tx >> 1;
        // ---- Jacobi in the position frame -------------------------------------------
        // Pair k always sits at positions (2k, 2k+1); after every step the positions
        // are permuted by the circle-method map (circ_next), so each sweep of tx-1
        // steps meets every index pair once.  H lives in packed upper-triangular form,
        // double buffered (read cur, write the permuted result to nxt), aliased onto
        // L0 (2 x 528 complex = one 32x33 tile).  Q stays in the original (label)
        // order; Lab[.][p] is the label at position p.  All addressing is static per
        // thread, so a step is branch-free with one barrier.
        __shared__ int Lab[2][TXMAX];
        __shared__ double4 RotS[TXMAX / 2];
        {
            const int j = t & 31, i0 = t >> 5;  // rows i0, i0+8, i0+16, i0+24 of column j
            const d2 h0 = L0[i0 * HS + j], h1 = L0[(i0 + 8) * HS + j];
            const d2 h2 = L0[(i0 + 16) * HS + j], h3 = L0[(i0 + 24) * HS + j];
            __syncthreads();
            if (i0 <= j) L0[up_idx(i0, j)] = h0;
            if (i0 + 8 <= j) L0[up_idx(i0 + 8, j)] = h1;
            if (i0 + 16 <= j) L0[up_idx(i0 + 16, j)] = h2;
            if (i0 + 24 <= j) L0[up_idx(i0 + 24, j)] = h3;
            if (t < TXMAX) Lab[0][t] = t;
            __syncthreads();
        }
        d2* Hp = L0;                              // Hp[buf * 528 + up_idx(i, j)]
        // static per-thread block (ta <= tb): read / write slots, conj flags
        int ta = -1, tb = -1;
        if (t < 136) {
            ta = c_tri_a[t];
            tb = c_tri_b[t];
            if (tb >= P) ta = -1;
        }
        const int sa = ta < 0 ? 0 : ta, sb = tb < 0 ? 0 : tb;
        int rd[4], wr[4], dg[4], dgj[4];
        double wsg[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 2 * sa + (r >> 1), j = 2 * sb + (r & 1);
            rd[r] = i <= j ? up_idx(i, j) : up_idx(j, i);
            dg[r] = up_idx(i, i);   // diagonals of row i and column j (convergence test)
            dgj[r] = up_idx(j, j);
            const int ii = circ_next(tx, i), jj = circ_next(tx, j);
            wr[r] = ii <= jj ? up_idx(ii, jj) : up_idx(jj, ii);
            wsg[r] = ii <= jj ? 1.0 : -1.0;
        }
        const bool diagblk = (ta == tb);                // (2k+1, 2k) mirrors (2k, 2k+1): not stored
        const double rsg10 = diagblk ? -1.0 : 1.0;      // diagonal block reads (2k+1,2k) as conj
        const int kl = lane & 15;                       // rotation evaluated by this lane
        const int rp = up_idx(2 * kl, 2 * kl), rq = up_idx(2 * kl + 1, 2 * kl + 1), rc = up_idx(2 * kl, 2 * kl + 1);
        const int pn = t < tx ? circ_next(tx, t) : 0;
        int cur = 0, sweeps = 0;
#ifdef ACE_DEBUG_SWEEPS
        dbg_t1 = __builtin_amdgcn_s_memrealtime();
#endif
        for (; sweeps < MAX_SWEEPS; ++sweeps) {
            // convergence pre-check over this thread's block entries (off-diagonal ones)
            if (ta >= 0) {
                const d2* H = Hp + cur * 528;
                bool need = false;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const bool offd = !diagblk || r == 1;   // off-diagonal entries of the block
                    if (offd) need |= needs_rot(H[dg[r]].x, H[dgj[r]].x, H[rd[r]], abs_tol);
                }
                if (need) flags[sweeps] = 1;
            }
            __syncthreads();
            if (!flags[sweeps]) break;
            for (int s = 0; s < tx - 1; ++s) {
                const int nx = cur ^ 1;
                const d2* H = Hp + cur * 528;
                d2* Hn = Hp + nx * 528;
                // rotations of the step, once per work-group (wave 0, lanes 0..P-1)
                if (t < P) {
                    const Rot J = make_rot(H[rp].x, H[rq].x, H[rc], abs_tol);
                    RotS[t] = make_double4(J.cs, J.sn, J.e.x, J.e.y);
                }
                __syncthreads();
                const double4 ra = RotS[sa], rb = RotS[sb], rl = RotS[kl];
                Rot Ja, Jb, Jl;
                Ja.cs = ra.x; Ja.sn = ra.y; Ja.e = make_double2(ra.z, ra.w);
                Jb.cs = rb.x; Jb.sn = rb.y; Jb.e = make_double2(rb.z, rb.w);
                Jl.cs = rl.x; Jl.sn = rl.y; Jl.e = make_double2(rl.z, rl.w);
                if (ta >= 0) {
                    // H'[a,b] = Ja^H H[a,b] Jb,  J = [[cs, sn], [-sn e*, cs e*]]
                    const d2 h00 = H[rd[0]], h01 = H[rd[1]], h11 = H[rd[3]];
                    d2 h10 = H[rd[2]];
                    h10.y *= rsg10;
                    const d2 ebc = make_double2(Jb.e.x, -Jb.e.y);
                    const d2 t01 = cmul(h01, ebc), t11 = cmul(h11, ebc);
                    const d2 T00 = csub(cscale(h00, Jb.cs), cscale(t01, Jb.sn));
                    const d2 T01 = cadd(cscale(h00, Jb.sn), cscale(t01, Jb.cs));
                    const d2 T10 = csub(cscale(h10, Jb.cs), cscale(t11, Jb.sn));
                    const d2 T11 = cadd(cscale(h10, Jb.sn), cscale(t11, Jb.cs));
                    const d2 u10 = cmul(Ja.e, T10), u11 = cmul(Ja.e, T11);
                    const d2 nv[4] = {csub(cscale(T00, Ja.cs), cscale(u10, Ja.sn)),
                                      csub(cscale(T01, Ja.cs), cscale(u11, Ja.sn)),
                                      cadd(cscale(T00, Ja.sn), cscale(u10, Ja.cs)),
                                      cadd(cscale(T01, Ja.sn), cscale(u11, Ja.cs))};
                    Hn[wr[0]] = make_double2(nv[0].x, nv[0].y * wsg[0]);
                    Hn[wr[1]] = make_double2(nv[1].x, nv[1].y * wsg[1]);
                    Hn[wr[3]] = make_double2(nv[3].x, nv[3].y * wsg[3]);
                    if (!diagblk) Hn[wr[2]] = make_double2(nv[2].x, nv[2].y * wsg[2]);
                }
                // Q <- Q J on label columns (Lab[2k], Lab[2k+1]) for (row i, pair k = lane & 15)
                if (kl < P) {
                    const int lp = Lab[cur][2 * kl], lq = Lab[cur][2 * kl + 1];
                    const d2 ebc = make_double2(Jl.e.x, -Jl.e.y);
#pragma unroll
                    for (int e = t; e < TXMAX * 16; e += 256) {
                        const int i = e >> 4;
                        if (i < tx) {
                            const d2 qp = L1[i * HS + lp];
                            const d2 qq = cmul(L1[i * HS + lq], ebc);
                            L1[i * HS + lp] = csub(cscale(qp, Jl.cs), cscale(qq, Jl.sn));
                            L1[i * HS + lq] = cadd(cscale(qp, Jl.sn), cscale(qq, Jl.cs));
                        }
                    }
                }
                if (t < tx) Lab[nx][pn] = Lab[cur][t];
                cur = nx;
                __syncthreads();
            }
        }
        if (sweeps >= MAX_SWEEPS && t == 0) atomicOr(&st->status, (int)ACE_ST_EIG_NOCONV);
#ifdef ACE_DEBUG_SWEEPS
        dbg_t2 = __builtin_amdgcn_s_memrealtime();
#endif
        // eigenvalue at position p belongs to eigenvector (Q column) Lab[p]
        if (t < tx) wv[Lab[cur][t]] = Hp[cur * 528 + up_idx(t, t)].x;
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
        }
        if (t < TXMAX) scl[t] = 1.0;
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
        if (a.Q) {
            for (int e = t; e < tx * tx; e += nt) Qg[e] = L1[(e / tx) * HS + (e % tx)];
        }
        if (flag_any) {
            // Z = U diag(sqrt(scl)) U^H E  (:482-484); E restaged into L0
            for (int e = t; e < TXMAX * TXMAX; e += nt) {
                const int i = e & 31, j = e >> 5;
                L0[i * HS + j] = (i < tx && j < rx) ? evalE(i + tx * j) : make_double2(0.0, 0.0);
            }
            __syncthreads();
            mm32<true, false>(L1, L0, cr, ci, lane, w);   // U^H E
#pragma unroll
            for (int r = 0; r < 4; ++r) {                 // row c of the product is eigen index c
                const double sw = sqrt(scl[16 * (w >> 1) + (lane >> 4) + 4 * r]);
                cr[r] *= sw;
                ci[r] *= sw;
            }
            __syncthreads();
            store32(L0, cr, ci, lane, w);
            __syncthreads();
            mm32<false, false>(L1, L0, cr, ci, lane, w);  // U (diag(sqrt(scl)) U^H E)
            __syncthreads();
            store32(L0, cr, ci, lane, w);
            __syncthreads();
            for (int k = t; k < n; k += nt) emit(k, L0[(k % tx) * HS + k / tx]);
        } else {
            for (int k = t; k < n; k += nt) emit(k, evalE(k));
        }
#ifdef ACE_DEBUG_SWEEPS
        __syncthreads();
        const unsigned long long dbg_t3 = __builtin_amdgcn_s_memrealtime();
        if (t == 0 && (b == 0 || b == 2000) && (a.it < 4 || a.it % 20 == 0))
            printf("b %d it %d sweeps %d pre %llu jac %llu post %llu (x10ns)\n", b, a.it, sweeps, dbg_t1 - dbg_t0,
                   dbg_t2 - dbg_t1, dbg_t3 - dbg_t2);
#endif
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
    if (t == 0) flag_improved = iter_control(a, st, mu, v6[0], v6[1], v6[2], v6[3], v6[4], v6[5]);
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

// ACE_ZSTEP_4WAVE=1 selects the four-wave A2only kernel above (A/B comparisons).
static bool use_4wave_zstep() {
    static const bool v = [] {
        const char* e = getenv("ACE_ZSTEP_4WAVE");
        return e && e[0] == '1';
    }();
    return v;
}

void launch_zstep(int variant, bool init, const ZArgs& a, int batch, hipStream_t st) {
    if (variant == ACE_VARIANT_NUCLEAR) {
        if (init) hipLaunchKernelGGL((zstep_kernel<ACE_VARIANT_NUCLEAR, true>), dim3(batch), dim3(256), 0, st, a);
        else hipLaunchKernelGGL((zstep_kernel<ACE_VARIANT_NUCLEAR, false>), dim3(batch), dim3(256), 0, st, a);
    } else if (!use_4wave_zstep()) {
        launch_zstep1w(init, a, batch, st);
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
