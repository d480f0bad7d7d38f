// Per-realisation kernels of the ADMM iteration (one work-group per realisation):
//   pre   : V = Z - N/mu, S = Y - M/mu                       (operands of ArgMinX)
//   ystep : AX = S - g, ArgMinY, M update, m-space reductions (inferLowRankV4_multi.m:329,:336-337,:345)
//   zstep : ArgMinZ (A2only spectral tail rescale via a Hermitian Jacobi eigensolver
//           of the tx x tx matrix E E^H in LDS; nuclear: singular-value soft threshold),
//           N update, residuals, convergence test, best-objective tracking, mu update
//           (:333, :340-341, :344-382)
// The four-wave zstep handles any column count r (the r = 20 stages of
// inferLowRankImpl, :258/:270, and the r = 1 refinement); the one-wave kernel of
// ace_zprox1w.hip is the fast A2only path at r = 1.
//
// ArgMinX runs in Woodbury form.  With G = (I + A A^H)^{-1} and K = A A^H:
//   inv(A^H A + I) (A^H s + v) = v + A^H G (s - A v),     A X = s - G (s - A v),
//   ||A^H d||^2 = d^H K d.
// This is algebraically identical to the reference's X = U (A'(Y-M/mu) + Z-N/mu)
// (:325, ArgMinX :404) and to its A'*Y residual terms (:330, :365, :369); it
// replaces the n x n apply by m x m ones.
#include "ace_common.hpp"
#include "ace_zcommon.hpp"
#include "ace_eig.hpp"
#include "ace_topk.hpp"

namespace ace {

namespace {
constexpr int TXMAX = 32;
constexpr int HS = ZHS;  // LDS row stride (complex) for 32x32 tiles

// GRAM (nuclear only): r > 1, singular values through the r x r Gram matrix.
template <int VARIANT, bool INIT, bool GRAM>
__global__ __launch_bounds__(256) void zstep_kernel(ZArgs a) {
    const int b = blockIdx.x;
    const int t = threadIdx.x, nt = blockDim.x, lane = t & 63, w = t >> 6;
    const int n = a.n, m = a.m, tx = a.tx, rx = a.rx, r = a.r;
    const int rn = r * n;
    RealState* st = a.st + b;
    __shared__ double red[16 * 8];
    __shared__ int flag_improved, flag_any;
    if (!INIT && st->done) return;
    const double mu = INIT ? 1.0 : st->mu;
    const double imu = 1.0 / mu;
    const d2* X = reinterpret_cast<const d2*>(a.X) + (long long)b * rn;
    d2* N = reinterpret_cast<d2*>(a.N) + (long long)b * rn;
    d2* Z = reinterpret_cast<d2*>(a.Z) + (long long)b * rn;

    // The r-column A2only stages keep N as exact zero after a Z-step with Z = E (no tail rescaling), as the
    // unit path does (RealState::nzero, ace_zprox1w.hip): N + mu (X - E) is zero up to the rounding of
    // E = X + N/mu.  While it holds, N is neither read nor written here, nor read by the applies of the next
    // iteration (i8a, i8ah's X = Z - N/mu + W, pre_kernel): they take the zero vector.
    const bool nzr = !INIT && VARIANT == ACE_VARIANT_A2ONLY && r > 1;
    const bool nz_in = nzr && st->nzero;
    const d2 zero2 = make_double2(0.0, 0.0);
    // accumulators: nX2, nZ2, nJN2, dZ2
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    VMax vz, vn;   // max |Z|, |N| of the outputs: the next apply's bound on |Z - N/mu|
    auto emit_pre = [&](int k, d2 znew, d2 x, d2 zo, d2 nold) {  // per-element update + reductions
        vz.add(znew);
        if (!INIT) {
            const d2 d = csub(x, znew);
            const d2 nnew = cadd(nold, cscale(d, mu));
            N[k] = nnew;
            vn.add(nnew);
            acc[0] += cabs2(x);
            acc[1] += cabs2(znew);
            acc[2] += cabs2(d);
            acc[3] += cabs2(csub(znew, zo));
        }
        Z[k] = znew;
    };
    // zeq: Z = E (no rescaling) -- with nzr the new N is the exact zero vector (not stored)
    auto emit = [&](int k, d2 znew, bool zeq = false) {  // per-element update + reductions
        const d2 x = X[k];
        vz.add(znew);
        if (!INIT) {
            const d2 zo = Z[k];
            const d2 d = csub(x, znew);
            if (!(nzr && zeq)) {
                const d2 nnew = cadd(nz_in ? zero2 : N[k], cscale(d, mu));
                N[k] = nnew;
                vn.add(nnew);
            }
            acc[0] += cabs2(x);
            acc[1] += cabs2(znew);
            acc[2] += cabs2(d);
            acc[3] += cabs2(csub(znew, zo));
        }
        Z[k] = znew;
    };
    auto evalE = [&](int k) -> d2 { return nz_in ? X[k] : cadd(X[k], cscale(N[k], imu)); };  // X + N/mu (:424)

    // The spectral branches use two 32x32 complex LDS tiles (operands / H in L0,
    // eigenvectors in L1); their 32x32 complex products run on the f64 matrix cores.
#define ACE_ZSTEP_LDS                         \
    __shared__ d2 L0[TXMAX * HS];             \
    __shared__ d2 L1[TXMAX * HS];             \
    __shared__ double wv[TXMAX], scl[TXMAX];  \
    __shared__ JacobiShared jsh;              \
    d4v cr, ci;

    if constexpr (VARIANT == ACE_VARIANT_NUCLEAR) {
        if constexpr (!GRAM) {
            // inferLowRank_Nuclear.m:411-419 at r = 1: Z = z * max(0, ||z|| - 1/mu) / ||z||
            double s[1] = {0.0};
            for (int k = t; k < n; k += nt) s[0] += cabs2(evalE(k));
            block_sum<1>(s, red);
            const double nz = sqrt(s[0]);
            const double f = nz > 0.0 ? fmax(0.0, nz - imu) / nz : 0.0;
            for (int k = t; k < n; k += nt) emit(k, cscale(evalE(k), f));
        } else {
            ACE_ZSTEP_LDS
            // Z = U soft(S, 1/mu) V^H of the n x r iterate (inferLowRank_Nuclear.m:411-439),
            // through its r x r Gram E^H E = V S^2 V^H:  Z = E V diag(max(0, s - 1/mu) / s) V^H.
            const int nch = (n + TXMAX - 1) / TXMAX;
            auto stage_rows = [&](int c) {  // L0[i][j] = E[32c + i][j], zero padded
                for (int e = t; e < TXMAX * TXMAX; e += nt) {
                    const int i = e & 31, j = e >> 5, row = TXMAX * c + i;
                    L0[i * HS + j] = (row < n && j < r) ? evalE(j * n + row) : make_double2(0.0, 0.0);
                }
            };
            cr = d4v{0.0, 0.0, 0.0, 0.0};
            ci = d4v{0.0, 0.0, 0.0, 0.0};
            for (int c = 0; c < nch; ++c) {
                stage_rows(c);
                __syncthreads();
                mm32_acc<true, false>(L0, L0, cr, ci, lane, w);  // += E_c^H E_c
                __syncthreads();
            }
            store32(L0, cr, ci, lane, w);
            for (int e = t; e < TXMAX * TXMAX; e += nt) L1[(e >> 5) * HS + (e & 31)] = make_double2((e >> 5) == (e & 31), 0.0);
            __syncthreads();
            const int sz = r + (r & 1);  // zero padded to an even order: the pad is an exact 0 eigenpair
            if (jacobi_eig32(L0, L1, sz, wv, jsh) >= JAC_MAX_SWEEPS && t == 0)
                atomicOr(&st->status, (int)ACE_ST_EIG_NOCONV);
            if (t < TXMAX) {
                const double s = t < sz ? sqrt(fmax(0.0, wv[t])) : 0.0;
                scl[t] = s > 0.0 ? fmax(0.0, s - imu) / s : 0.0;  // Shrink(S, 1/mu, 1) / S
            }
            __syncthreads();
            for (int e = t; e < TXMAX * TXMAX; e += nt) {  // L0 = diag(f) V^H
                const int c = e >> 5, i = e & 31;
                const d2 v = L1[i * HS + c];
                L0[c * HS + i] = make_double2(scl[c] * v.x, -scl[c] * v.y);
            }
            __syncthreads();
            mm32<false, false>(L1, L0, cr, ci, lane, w);    // W = V diag(f) V^H
            __syncthreads();
            store32(L1, cr, ci, lane, w);
            __syncthreads();
            for (int c = 0; c < nch; ++c) {
                stage_rows(c);
                __syncthreads();
                mm32<false, false>(L0, L1, cr, ci, lane, w);  // Z_c = E_c W
                __syncthreads();
                store32(L0, cr, ci, lane, w);
                __syncthreads();
                for (int e = t; e < TXMAX * TXMAX; e += nt) {
                    const int i = e & 31, j = e >> 5, row = TXMAX * c + i;
                    if (row < n && j < r) emit(j * n + row, L0[i * HS + j]);
                }
                __syncthreads();
            }
        }
    } else {
        // ---- A2only ArgMinZ (inferLowRankV4_multi.m:423-485) ------------------------
        // E = reshape(X + N/mu, tx, []) = [E_1 ... E_r], E_j = reshape(column j, tx, rx),
        // so E E^H = sum_j E_j E_j^H and Z_j = U diag(sqrt(scale)) U^H E_j.
        ACE_ZSTEP_LDS
        __shared__ double rs2[TXMAX];
        __shared__ int ord[TXMAX], ascp[TXMAX];
        const ZProfile pf = z_profile(a, b);
        // E_j (zero padded to 32 x 32) is fetched into registers one block ahead of its use, so
        // the loads of block j + 1 are in flight during block j's barrier and matrix-core step
        // (a barrier waits for LDS traffic only); 256 threads x 4 slots = one 32 x 32 tile.
        auto fetchE = [&](int j, d2 (&o)[4]) {
            const int base = j * n;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = t + 256 * u, i = e & 31, c = e >> 5;
                o[u] = (i < tx && c < rx) ? evalE(base + i + tx * c) : make_double2(0.0, 0.0);
            }
        };
        auto putE = [&](const d2 (&o)[4]) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = t + 256 * u;
                L0[(e & 31) * HS + (e >> 5)] = o[u];
            }
        };
        d2 eb[4];
        cr = d4v{0.0, 0.0, 0.0, 0.0};
        ci = d4v{0.0, 0.0, 0.0, 0.0};
#ifdef ACE_DEBUG_TK   // phase times of realisation 5 (10 ns units)
        unsigned long long zt[6];
        zt[0] = __builtin_amdgcn_s_memrealtime();
#endif
        const bool small = tx <= 16 && rx <= 16;
        const bool warm = (!INIT) && a.warm && a.Q;
        d2* Qg = a.Q ? reinterpret_cast<d2*>(a.Q) + (long long)b * tx * tx : nullptr;
        // H = E E^H into L0 (the warm frame Q^H H Q when warm), L1 = Q (or I): the Jacobi eigensolver's operands
        auto form_h = [&]() {
            cr = d4v{0.0, 0.0, 0.0, 0.0};
            ci = d4v{0.0, 0.0, 0.0, 0.0};
            // tx, rx <= 16 (the driver's 16 x 16 arrays): E E^H is one 16 x 16 tile, so each wave
            // accumulates the blocks j = w, w + 4, ... straight from memory (16 MFMAs per block, no
            // LDS staging or barrier per block) and the four partial tiles are summed in LDS.
            if (small) {
                for (int j = w; j < r; j += 4) {
                    d2 ev[4];
    #pragma unroll
                    for (int u = 0; u < 4; ++u) {   // lane: E_j[l & 15][4u + (l >> 4)]
                        const int i = lane & 15, kk = 4 * u + (lane >> 4);
                        ev[u] = (i < tx && kk < rx) ? evalE(j * n + i + tx * kk) : make_double2(0.0, 0.0);
                    }
    #pragma unroll
                    for (int u = 0; u < 4; ++u) {   // A = E_j, B = E_j^H: the lane's operands are e and conj(e)
                        const d2 av = ev[u];
                        cr = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, av.x, cr, 0, 0, 0);
                        cr = __builtin_amdgcn_mfma_f64_16x16x4f64(-av.y, -av.y, cr, 0, 0, 0);
                        ci = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, -av.y, ci, 0, 0, 0);
                        ci = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, av.x, ci, 0, 0, 0);
                    }
                }
                d2* part = L1;   // [4][16][16] partial tiles (exactly the L1 tile's 32 x 33 budget)
    #pragma unroll
                for (int rr = 0; rr < 4; ++rr)
                    part[w * 256 + ((lane >> 4) + 4 * rr) * 16 + (lane & 15)] = make_double2(cr[rr], ci[rr]);
                __syncthreads();
                for (int e = t; e < TXMAX * TXMAX; e += nt) {   // H (zero padded), waves summed in order
                    const int i = e >> 5, c = e & 31;
                    d2 h = make_double2(0.0, 0.0);
                    if (i < 16 && c < 16)
    #pragma unroll
                        for (int ww = 0; ww < 4; ++ww) h = cadd(h, part[ww * 256 + i * 16 + c]);
                    L0[i * HS + c] = h;
                }
                __syncthreads();
            } else {
                fetchE(0, eb);
                for (int j = 0; j < r; ++j) {
                    putE(eb);
                    if (j + 1 < r) fetchE(j + 1, eb);
                    __syncthreads();
                    mm32_acc<false, true>(L0, L0, cr, ci, lane, w);  // H += E_j E_j^H  (:428)
                    __syncthreads();
                }
                store32(L0, cr, ci, lane, w);
            }
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
                    const int rr = e >> 5, c = e & 31;
                    if (rr < c) {
                        const d2 u = L0[rr * HS + c], l = L0[c * HS + rr];
                        const d2 h = make_double2(0.5 * (u.x + l.x), 0.5 * (u.y - l.y));
                        L0[rr * HS + c] = h;
                        L0[c * HS + rr] = make_double2(h.x, -h.y);
                    } else if (rr == c) {
                        L0[rr * HS + c].y = 0.0;
                    }
                }
                __syncthreads();
            }
        };
        form_h();
#ifdef ACE_DEBUG_TK
        zt[1] = zt[0];
#endif
        // Ky Fan certificate (the one-wave kernel's): the sum of any r diagonal entries
        // of Q^H H Q (Q unitary: the warm start, or I) is at most the sum of the r largest
        // eigenvalues of H, so if the r_p largest diagonal entries clear f_p * trace with margin for
        // every profile entry, no tail rescaling fires (:475) and Z = E exactly (:482).  The
        // eigendecomposition is then skipped (Q stays the next warm start).
#ifdef ACE_DEBUG_TK
        zt[2] = __builtin_amdgcn_s_memrealtime();
#endif
        __shared__ int cert_s;
        if (t < tx) {   // descending order of the diagonal (ties by index)
            const double dk = L0[t * HS + t].x;
            int rank = 0;
            for (int j = 0; j < tx; ++j) {
                const double dj = L0[j * HS + j].x;
                rank += (dj > dk) || (dj == dk && j < t);
            }
            rs2[rank] = dk;
        }
        __syncthreads();
        if (t == 0) {
            double tr = 0.0;
            for (int k = 0; k < tx; ++k) tr += fmax(0.0, rs2[k]);
            int ok = tr > 0.0;
            #pragma unroll
            for (int pi = 0; pi < 4; ++pi) {
                if (pi >= pf.np) break;
                double vr = 0.0;
                for (int k = 0; k < pf.rl[pi]; ++k) vr += rs2[k];
                ok &= vr * (1.0 - 1e-12) > pf.fl[pi] * tr * (1.0 + 1e-9);
            }
            cert_s = a.zcert ? ok : 0;
        }
        __syncthreads();
        const bool cert = cert_s;
        if (cert) {
            if (t < TXMAX) scl[t] = 1.0;
            if (t == 0) flag_any = 0;
        } else {
        // the full profile's top-K eigenpairs by the one-wave tridiagonal reduction (topk_tri) in the cold
        // iterations (ZArgs::tkeig): wave 0 reduces H (packed into L1), the result R is the eigenbasis in the
        // warm frame (columns in descending order); a failed check forms H again for the Jacobi eigensolver
        bool tk = false;
        int maxr = 0;
#pragma unroll
        for (int pi = 0; pi < 4; ++pi) maxr = pi < pf.np ? max(maxr, pf.rl[pi]) : maxr;
        const int tkK = min(maxr, tx);
        if (a.tkeig > 0 && (INIT || a.it <= a.tkeig) && maxr <= TK_MAX && tx >= 2) {
            for (int e = t; e < TXMAX * TXMAX; e += nt) {
                const int i = e >> 5, c = e & 31;
                if (i <= c) L1[up_idx(i, c)] = L0[i * HS + c];
            }
            __syncthreads();
            __shared__ int tk_s;
            double* sd = reinterpret_cast<double*>(L0 + 32);   // topk_tri's scalars: 176 doubles
            if (w == 0) {
                const bool ok = topk_tri(L1, L0, sd, sd + 80, sd + 112, sd + 144, tx, tkK, lane, [] {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                });
                if (lane == 0) {
                    tk_s = ok;
                    if (a.tkcnt) atomicAdd(a.tkcnt + (ok ? 0 : 1), 1);
                }
            }
            __syncthreads();
            tk = tk_s;
            if (tk && t == 0) {
                // the rescale (:469-480) on the top-K eigenvalues and the tail as one sum (v = trace - top-K
                // sum; the one-wave kernel's rule): groups inside the top K their own factor, the tail the
                // common one
                const double* thk = sd + 64;
                double* s2 = wv;
                double tr = 0.0, top = 0.0;
                for (int k = 0; k < tx; ++k) tr += fmax(0.0, rs2[k]);
                for (int k = 0; k < tkK; ++k) {
                    s2[k] = fmax(0.0, thk[k]);
                    top += s2[k];
                }
                double tail = fmax(0.0, tr - top), stail = 1.0;
                for (int k = 0; k < TXMAX; ++k) scl[k] = 1.0;
                #pragma unroll
                for (int pi = 0; pi < 4; ++pi) {
                    if (pi >= pf.np) break;
                    const int rr = pf.rl[pi];
                    const double f = pf.fl[pi];
                    double vr = 0.0, v = 0.0;
                    for (int k = 0; k < tkK; ++k) {
                        if (k < rr) vr += s2[k];
                        v += s2[k];
                    }
                    v += tail;
                    if (vr < v * f) {
                        const double sc = fmin(1.0, vr / (v - vr) * (1.0 / f - 1.0));
                        for (int k = rr; k < tkK; ++k) {
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
            if (!tk) {
                form_h();
            } else if (warm) {   // the eigenbasis Q_prev R
                __syncthreads();
                for (int e = t; e < TXMAX * TXMAX; e += nt) {
                    const int i = e >> 5, c = e & 31;
                    L0[i * HS + c] = (i < tx && c < tx) ? Qg[i * tx + c] : make_double2(i == c ? 1.0 : 0.0, 0.0);
                }
                __syncthreads();
                mm32<false, false>(L0, L1, cr, ci, lane, w);
                __syncthreads();
                store32(L1, cr, ci, lane, w);
            }
            __syncthreads();
        }
        if (!tk) {
        if (jacobi_eig32(L0, L1, tx, wv, jsh) >= JAC_MAX_SWEEPS && t == 0)
            atomicOr(&st->status, (int)ACE_ST_EIG_NOCONV);
        ascending_positions(wv, tx, ascp);           // LAPACK order of eig (:428)
        if (t < tx) {  // stable descending rank of max(0, w) (:429-430)
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
            #pragma unroll  // constant trip count: the profile stays in registers
            for (int pi = 0; pi < 4; ++pi) {
                if (pi >= pf.np) break;
                const int rr = pf.rl[pi];
                const double f = pf.fl[pi];
                double vr = 0.0, v = 0.0;
                for (int k = 0; k < rr; ++k) vr += s2[k];
                for (int k = 0; k < tx; ++k) v += s2[k];
                if (vr < v * f) {
                    const double sc = fmin(1.0, vr / (v - vr) * (1.0 / f - 1.0));
                    for (int k = rr; k < tx; ++k) {
                        s2[k] *= sc;
                        scl[ord[k]] *= sc;
                    }
                }
            }
            int any = 0;
            for (int k = 0; k < tx; ++k) any |= scl[k] < 1.0;
            flag_any = any;
        }
        }   // !tk
        }
        __syncthreads();
#ifdef ACE_DEBUG_TK
        zt[3] = __builtin_amdgcn_s_memrealtime();
#endif
        if (a.Q && (!cert || !warm)) {   // (a certified cold step stores I: a unitary warm start)
            for (int e = t; e < tx * tx; e += nt) Qg[e] = L1[(e / tx) * HS + (e % tx)];
        }
        if (flag_any) {
            // W = U diag(sqrt(scl)) U^H (:482-484), then Z_j = W E_j for every block
            for (int e = t; e < TXMAX * TXMAX; e += nt) {  // L0 = diag(sqrt(scl)) U^H
                const int c = e >> 5, i = e & 31;
                const d2 u = L1[i * HS + c];
                const double sw = sqrt(scl[c]);
                L0[c * HS + i] = make_double2(sw * u.x, -sw * u.y);
            }
            __syncthreads();
            mm32<false, false>(L1, L0, cr, ci, lane, w);
            __syncthreads();
            store32(L1, cr, ci, lane, w);
            __syncthreads();
            if (small) {   // Z_j = W E_j per wave, block j = w, w + 4, ..., emitted from the MFMA outputs
                d2 wa[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) wa[u] = L1[(lane & 15) * HS + 4 * u + (lane >> 4)];   // A = W
                for (int j = w; j < r; j += 4) {
                    d2 ev[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {   // B = E_j: lane E_j[4u + (l >> 4)][l & 15]
                        const int kk = 4 * u + (lane >> 4), c = lane & 15;
                        ev[u] = (kk < tx && c < rx) ? evalE(j * n + kk + tx * c) : make_double2(0.0, 0.0);
                    }
                    d4v zr = d4v{0.0, 0.0, 0.0, 0.0}, zi = d4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const d2 av = wa[u], bv = ev[u];
                        zr = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.x, zr, 0, 0, 0);
                        zr = __builtin_amdgcn_mfma_f64_16x16x4f64(-av.y, bv.y, zr, 0, 0, 0);
                        zi = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.y, zi, 0, 0, 0);
                        zi = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bv.x, zi, 0, 0, 0);
                    }
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {   // lane l, reg rr -> Z_j[(l >> 4) + 4 rr][l & 15]
                        const int i = (lane >> 4) + 4 * rr, c = lane & 15;
                        if (i < tx && c < rx) emit(j * n + i + tx * c, make_double2(zr[rr], zi[rr]));
                    }
                }
            } else {
            // the emit inputs (X, old Z, old N) of block j are requested with block j + 1's E
            d2 px[4], pz[4], pn[4];
            auto fetchP = [&](int j) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = t + nt * u;
                    if (k < n) {
                        px[u] = X[j * n + k];
                        pz[u] = INIT ? make_double2(0.0, 0.0) : Z[j * n + k];
                        pn[u] = nz_in ? zero2 : N[j * n + k];
                    }
                }
            };
            fetchE(0, eb);
            fetchP(0);
            for (int j = 0; j < r; ++j) {
                putE(eb);
                if (j + 1 < r) fetchE(j + 1, eb);
                __syncthreads();
                mm32<false, false>(L1, L0, cr, ci, lane, w);  // W E_j
                __syncthreads();
                store32(L0, cr, ci, lane, w);
                __syncthreads();
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = t + nt * u;
                    if (k < n) emit_pre(j * n + k, L0[(k % tx) * HS + k / tx], px[u], pz[u], pn[u]);
                }
                if (j + 1 < r) fetchP(j + 1);
                __syncthreads();
            }
            }
        } else {
            // Z = E: the element stream in batches of 4 per thread, loads issued before the stores
            for (int k0 = 0; k0 < rn; k0 += 4 * nt) {
                d2 ev[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = k0 + t + nt * u;
                    ev[u] = k < rn ? evalE(k) : make_double2(0.0, 0.0);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = k0 + t + nt * u;
                    if (k < rn) emit(k, ev[u], true);
                }
            }
        }
#ifdef ACE_DEBUG_TK
        zt[4] = __builtin_amdgcn_s_memrealtime();
        if (t == 0 && (b == 5 || b == 700) && r > 1)
            printf("zs4 b %d it %d r %d: H %llu warm %llu eig(cert %d) %llu W+Z %llu (x10ns)\n", b, a.it, r, zt[1] - zt[0],
                   zt[2] - zt[1], (int)cert, zt[3] - zt[2], zt[4] - zt[3]);
#endif
    }
#undef ACE_ZSTEP_LDS
    if constexpr (VARIANT == ACE_VARIANT_A2ONLY) {
        if (nzr && t == 0) st->nzero = flag_any ? 0 : 1;
    }
    // bound for the next iteration's V = Z - N/mu (written after iter_control's mu update)
    double vb[3] = {wave_max(vz.m), wave_max(vn.m), wave_sum(vz.s + vn.s)};
    __syncthreads();
    if (lane == 0) {
        red[64 + 3 * w] = vb[0];
        red[64 + 3 * w + 1] = vb[1];
        red[64 + 3 * w + 2] = vb[2];
    }
    __syncthreads();
    if (t == 0)
        for (int k = 1; k < nt / 64; ++k) {
            vb[0] = fmax(vb[0], red[64 + 3 * k]);
            vb[1] = fmax(vb[1], red[64 + 3 * k + 1]);
            vb[2] += red[64 + 3 * k + 2];
        }
    auto write_vbound = [&]() {
        if (t == 0) st->vbound = (vb[0] + vb[1] * (1.0 / st->mu)) * (1.0 + 0x1p-40) + vb[2];
    };
    if (INIT) {
        write_vbound();
        return;
    }

    // m-space dual terms: ||A^H (Y - Y0)||^2 = dY^H (K Y - K Y0),  ||A^H Y||^2 = Y^H K Y
    const int rm = r * m;
    double v6[6] = {acc[0], acc[1], acc[2], acc[3], 0.0, 0.0};
    {
        const d2* Yn = reinterpret_cast<const d2*>(a.Ynew) + (long long)b * rm;
        const d2* Yo = reinterpret_cast<const d2*>(a.Yold) + (long long)b * rm;
        const d2* Kn = reinterpret_cast<const d2*>(a.KYnew) + (long long)b * rm;
        const d2* Ko = reinterpret_cast<const d2*>(a.KYold) + (long long)b * rm;
        for (int i = t; i < rm; i += nt) {
            const d2 yn = Yn[i], kn = Kn[i];
            const d2 dy = csub(yn, Yo[i]), dk = csub(kn, Ko[i]);
            v6[4] += dy.x * dk.x + dy.y * dk.y;
            v6[5] += yn.x * kn.x + yn.y * kn.y;
        }
    }
    block_sum<6>(v6, red);
#ifdef ACE_DEBUG_SPEC
    if (t == 0 && b == 0 && a.it <= 4)
        printf("zstep v%d r %d it %d mu %g obj2 %g nAX2 %g nY2 %g | nX2 %g nZ2 %g jn2 %g dZ2 %g dAtY %g nAtY %g\n", VARIANT, r,
               a.it, mu, st->obj2, st->nAX2, st->nY2, v6[0], v6[1], v6[2], v6[3], v6[4], v6[5]);
#endif
    if (t == 0) flag_improved = iter_control(a, st, mu, v6[0], v6[1], v6[2], v6[3], v6[4], v6[5]) & 1;   // (no lazy_dual here)
    write_vbound();
    __syncthreads();
    if (flag_improved) {  // best-objective iterate (:344-361): all columns, or the argmin column
        const d2* Yn = reinterpret_cast<const d2*>(a.Ynew) + (long long)b * rm;
        const int c0 = a.row_mode ? 0 : st->objcol, nc = a.row_mode ? r : 1;
        d2* oX = reinterpret_cast<d2*>(a.optX) + (long long)b * nc * n;
        d2* oY = reinterpret_cast<d2*>(a.optY) + (long long)b * nc * m;
        for (int k = t; k < nc * n; k += nt) oX[k] = X[c0 * n + k];
        for (int i = t; i < nc * m; i += nt) oY[i] = Yn[c0 * m + i];
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
    if (Vp) {   // (the int8 r-column stages form V inside their applies: S only)
        d2* V = reinterpret_cast<d2*>(Vp) + (long long)b * n;
        const bool nz = st[b].nzero;   // (N held as exact zero: the r-column stages, zstep_kernel)
        for (int k = threadIdx.x; k < n; k += blockDim.x) V[k] = nz ? Z[k] : csub(Z[k], cscale(N[k], imu));
    }
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
        const d2 mi = M[i];
        // S == null: S = Y - M/mu is formed here (pre_kernel folded into the GEMMs)
        const d2 si = Sp ? S[i] : csub(Yo[i], cscale(mi, imu));
        const d2 ax = csub(si, g[i]);
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

// the one-wave A2only kernel forms X from W = A^H g itself (ZArgs::wmode)
bool zstep_takes_w(int variant, int r) {
    (void)variant;   // A2only and A2nuclear (r = 1) both run the one-wave kernel
    return r == 1 && !use_4wave_zstep();
}

void launch_zstep(int variant, bool init, const ZArgs& a, int batch, hipStream_t st) {
#define ACE_ZL(V, I, G) hipLaunchKernelGGL((zstep_kernel<V, I, G>), dim3(batch), dim3(256), 0, st, a)
    if (variant == ACE_VARIANT_NUCLEAR && a.r == 1 && !use_4wave_zstep()) {
        launch_zstep1w(init, a, batch, st);   // ZArgs::nuclear selects the soft threshold
    } else if (variant == ACE_VARIANT_NUCLEAR) {
        if (a.r == 1) {
            if (init) ACE_ZL(ACE_VARIANT_NUCLEAR, true, false);
            else ACE_ZL(ACE_VARIANT_NUCLEAR, false, false);
        } else {
            if (init) ACE_ZL(ACE_VARIANT_NUCLEAR, true, true);
            else ACE_ZL(ACE_VARIANT_NUCLEAR, false, true);
        }
    } else if (a.r == 1 && !use_4wave_zstep()) {
        launch_zstep1w(init, a, batch, st);
    } else {
        if (init) ACE_ZL(ACE_VARIANT_A2ONLY, true, false);
        else ACE_ZL(ACE_VARIANT_A2ONLY, false, false);
    }
#undef ACE_ZL
}
// Shrink (inferLowRank_Nuclear.m:421-439) of the n x r matrices E_b on their own: the init form of
// the GRAM nuclear Z-step (mu = 1, N = 0, threshold 1) on E / tau, scaled back by tau
// (exact for a power-of-two tau).  Columns of E_b are contiguous ([b][r][n]).
__global__ void scale_kernel(long long cnt, double f, const double* __restrict__ x, double* __restrict__ y) {
    const long long i = blockIdx.x * 256LL + threadIdx.x;
    if (i < cnt) y[i] = x[i] * f;
}
int launch_nuclear_prox(int batch, int n, int r, const double* E, double tau, double* Zo, hipStream_t st) {
    const long long cnt = 2LL * batch * r * n;
    double *X = nullptr, *N = nullptr;
    RealState* rs = nullptr;
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&X), sizeof(double) * cnt, st);
    if (e == hipSuccess) e = hipMallocAsync(reinterpret_cast<void**>(&N), sizeof(double) * cnt, st);
    if (e == hipSuccess) e = hipMallocAsync(reinterpret_cast<void**>(&rs), sizeof(RealState) * batch, st);
    if (e == hipSuccess) e = hipMemsetAsync(N, 0, sizeof(double) * cnt, st);
    if (e == hipSuccess) e = hipMemsetAsync(rs, 0, sizeof(RealState) * batch, st);
    if (e == hipSuccess) {
        const unsigned gb = (unsigned)((cnt + 255) / 256);
        if (tau == 1.0) e = hipMemcpyAsync(X, E, sizeof(double) * cnt, hipMemcpyDeviceToDevice, st);
        else hipLaunchKernelGGL(scale_kernel, dim3(gb), dim3(256), 0, st, cnt, 1.0 / tau, E, X);
        ZArgs a{};
        a.n = n;
        a.r = r;
        a.tx = n;
        a.rx = 1;
        a.X = X;
        a.N = N;
        a.Z = Zo;
        a.st = rs;
        hipLaunchKernelGGL((zstep_kernel<ACE_VARIANT_NUCLEAR, true, true>), dim3(batch), dim3(256), 0, st, a);
        if (tau != 1.0) hipLaunchKernelGGL(scale_kernel, dim3(gb), dim3(256), 0, st, cnt, tau, Zo, Zo);
        if (e == hipSuccess) e = hipGetLastError();
    }
    if (X) (void)hipFreeAsync(X, st);
    if (N) (void)hipFreeAsync(N, st);
    if (rs) (void)hipFreeAsync(rs, st);
    return e == hipSuccess ? 0 : (int)e;
}
void launch_pre(int n, int m, int batch, const double* Z, const double* N, const double* Y, const double* M, double* V,
                double* S, const RealState* rs, hipStream_t st) {
    hipLaunchKernelGGL(pre_kernel, dim3(batch), dim3(256), 0, st, n, m, Z, N, Y, M, V, S, rs);
}
void launch_ystep(int m, int batch, const double* S, const double* g, double* M, const double* B, const double* Yold,
                  double* Ynew, RealState* rs, hipStream_t st) {
    hipLaunchKernelGGL(ystep_kernel, dim3(batch), dim3(256), 0, st, m, S, g, M, B, Yold, Ynew, rs);
}
void launch_conj_transpose(int rows, int cols, const double* A, double* AH, hipStream_t st) {
    dim3 grid((cols + 31) / 32, (rows + 31) / 32);
    hipLaunchKernelGGL(conj_transpose_kernel, grid, dim3(256), 0, st, rows, cols, A, AH);
}

}  // namespace ace
