// Kernels of the r-column ADMM stages and of the recovery pipeline around them
// (main/src/my_recovery_algorithms/ADMM_v2/inferLowRankV4_multi.m).  One work-group
// per realisation unless stated; per-realisation state is column-major per
// realisation: X[b][j][n], Y[b][j][m] (column j of the n x r / m x r iterate is
// contiguous, so the GEMMs see batch*r independent vectors).
//
//   init_r      InferADMM init :296-310 (row mode :301, column mode :303-305,
//               normalize_rows :538-559)
//   ystep_r     ArgMinY :511-533 + M update :336-337 + the m-space reductions;
//               column mode also the per-column objective and its first argmin :352-361
//   finalize_r  opt_X / opt_Y (:384-385)
//   pipeline    normalisation :27-38, train/test gathers :48-53, the rotation by the
//               eigenvectors of X^H X :263-264, test quality :68, best-of-restarts
//               :79-83, rollback :93-98 and rescale :106-107
#include "ace_common.hpp"
#include "ace_eig.hpp"
#include "ace_pipe.hpp"

namespace ace {

namespace {
constexpr int RMAX = 32;  // max columns per realisation (r = min(20, m, n) in the reference)

template <bool ROW>
__global__ __launch_bounds__(256) void init_r_kernel(int n, int m, int r, const double* X0p, const double* P0p,
                                                     const double* Bp, double* Xp, double* Yp, double* Mp,
                                                     double* Np, RealState* st, double mu0, const unsigned char* maskp,
                                                     int ldmask) {
    const int b = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    // per-realisation train rows in m-space (PartRows): test rows take no part and stay Y = M = 0
    const unsigned char* mask = maskp ? maskp + (long long)b * ldmask : nullptr;
    __shared__ double red[16 * (1 + RMAX)];
    __shared__ double scale[RMAX];
    const long long rn = (long long)r * n, rm = (long long)r * m;
    const d2* X0 = reinterpret_cast<const d2*>(X0p) + b * rn;
    const d2* P0 = reinterpret_cast<const d2*>(P0p) + b * rm;
    const double* B = Bp + (long long)b * m;
    double v[1 + RMAX];
#pragma unroll
    for (int j = 0; j <= RMAX; ++j) v[j] = 0.0;
    for (int i = t; i < m; i += nt) {
        if (mask && !mask[i]) continue;
        v[0] += B[i] * B[i];
#pragma unroll
        for (int j = 0; j < RMAX; ++j)
            if (j < r) v[1 + j] += cabs2(P0[j * m + i]);
    }
    block_sum<1 + RMAX>(v, red);
    const double nB = sqrt(v[0]);
    if (t < r) {
        double s2 = 0.0;  // (static register indexing: loops over RMAX)
        if (ROW) {  // :301  X * (norm(B) / norm(AX, 'fro'))
#pragma unroll
            for (int j = 0; j < RMAX; ++j) s2 += (j < r) ? v[1 + j] : 0.0;
        } else {    // :303-305  per column
#pragma unroll
            for (int j = 0; j < RMAX; ++j) s2 = (j == t) ? v[1 + j] : s2;
        }
        scale[t] = nB / sqrt(s2);
    }
    __syncthreads();
#ifdef ACE_DEBUG_SPEC
    if (t == 0 && b == 0) printf("init_r r %d m %d n %d nB %g scale0 %g scale1 %g P0sq0 %g\n", r, m, n, nB, scale[0], r > 1 ? scale[1] : 0.0, v[1]);
#endif
    d2* X = reinterpret_cast<d2*>(Xp) + b * rn;
    d2* N = reinterpret_cast<d2*>(Np) + b * rn;
    for (long long k = t; k < rn; k += nt) {
        X[k] = cscale(X0[k], scale[k / n]);
        N[k] = make_double2(0.0, 0.0);
    }
    // Y = normalize_rows(A X, B)  (A X = scale * P0)
    d2* Y = reinterpret_cast<d2*>(Yp) + b * rm;
    d2* M = reinterpret_cast<d2*>(Mp) + b * rm;
    const double isr = 1.0 / sqrt((double)r);
    for (int i = t; i < m; i += nt) {
        const double bi = B[i];
        if (mask && !mask[i]) {
            for (int j = 0; j < r; ++j) Y[j * m + i] = M[j * m + i] = make_double2(0.0, 0.0);
            continue;
        }
        if (ROW) {
            double d2s = 0.0;
            for (int j = 0; j < r; ++j) d2s += cabs2(cscale(P0[j * m + i], scale[j]));
            const double D = sqrt(d2s);
            for (int j = 0; j < r; ++j) {
                const d2 ax = cscale(P0[j * m + i], scale[j]);
                Y[j * m + i] = D == 0.0 ? make_double2(isr * bi, 0.0) : cscale(ax, bi / D);
                M[j * m + i] = make_double2(0.0, 0.0);
            }
        } else {
            for (int j = 0; j < r; ++j) {
                const d2 ax = cscale(P0[j * m + i], scale[j]);
                const double D = sqrt(cabs2(ax));
                Y[j * m + i] = D == 0.0 ? make_double2(bi, 0.0) : cscale(ax, bi / D);
                M[j * m + i] = make_double2(0.0, 0.0);
            }
        }
    }
    if (t == 0) {
        RealState s = {};
        s.mu = mu0;
        s.last_res = INFINITY;
        s.opt_obj = INFINITY;
        s.nB = nB;
        st[b] = s;
    }
}

// AX = S - g, C = AX + M/mu; row mode: Y_i = C_i (B_i/||C_i|| + mu)/(1 + mu) (zero row ->
// 1/sqrt(r)); column mode: entrywise with |C_ij| (zero -> 1).  M += mu (AX - Y).
template <bool ROW>
__global__ __launch_bounds__(256) void ystep_r_kernel(int m, int r, const double* Sp, const double* gp, double* Mp,
                                                      const double* Bp, const double* Yold, double* Ynew,
                                                      RealState* st, const unsigned char* maskp, int ldmask) {
    constexpr int NV = ROW ? 5 : 5 + RMAX;
    const int b = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    const unsigned char* mask = maskp ? maskp + (long long)b * ldmask : nullptr;   // (as init_r_kernel)
    __shared__ double red[16 * NV];
    if (st[b].done) return;
    const double mu = st[b].mu, imu = 1.0 / mu;
    const long long rm = (long long)r * m;
    const d2* S = reinterpret_cast<const d2*>(Sp) + b * rm;
    const d2* g = reinterpret_cast<const d2*>(gp) + b * rm;
    d2* M = reinterpret_cast<d2*>(Mp) + b * rm;
    const double* B = Bp + (long long)b * m;
    const d2* Yo = reinterpret_cast<const d2*>(Yold) + b * rm;
    d2* Yn = reinterpret_cast<d2*>(Ynew) + b * rm;
    double v[NV];  // obj2 (row mode), nAX2, nY2, nJM2, dY2, per-column obj2 (column mode)
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = 0.0;
    const double isr = 1.0 / sqrt((double)r);
    auto finish = [&](int e, d2 ax, d2 y) {
        const d2 jm = csub(ax, y);
        M[e] = cadd(M[e], cscale(jm, mu));
        v[1] += cabs2(ax);
        v[2] += cabs2(y);
        v[3] += cabs2(jm);
        v[4] += cabs2(csub(y, Yo[e]));
        Yn[e] = y;
    };
    for (int i = t; i < m; i += nt) {
        const double bi = B[i];
        if (mask && !mask[i]) {
            for (int j = 0; j < r; ++j) Yn[j * m + i] = make_double2(0.0, 0.0);
            continue;
        }
        if constexpr (ROW) {
            double d2s = 0.0, ax2 = 0.0;
            for (int j = 0; j < r; ++j) {
                const int e = j * m + i;
                const d2 ax = csub(S[e], g[e]);
                d2s += cabs2(cadd(ax, cscale(M[e], imu)));
                ax2 += cabs2(ax);
            }
            const double D = sqrt(d2s);
            const bool zero = D == 0.0;
            const double f = (bi / (zero ? 1.0 : D) + mu) / (1.0 + mu);
            for (int j = 0; j < r; ++j) {
                const int e = j * m + i;
                const d2 ax = csub(S[e], g[e]);
                const d2 c = zero ? make_double2(isr, 0.0) : cadd(ax, cscale(M[e], imu));
                finish(e, ax, cscale(c, f));
            }
            const double o = sqrt(ax2) - bi;
            v[0] += o * o;
        } else {
#pragma unroll
            for (int j = 0; j < RMAX; ++j) {
                if (j < r) {
                    const int e = j * m + i;
                    const d2 ax = csub(S[e], g[e]);
                    d2 c = cadd(ax, cscale(M[e], imu));
                    double D = sqrt(cabs2(c));
                    if (D == 0.0) {
                        c = make_double2(1.0, 0.0);
                        D = 1.0;
                    }
                    finish(e, ax, cscale(c, (bi / D + mu) / (1.0 + mu)));
                    const double o = sqrt(cabs2(ax)) - bi;
                    v[5 + j] += o * o;
                }
            }
        }
    }
    block_sum<NV>(v, red);
    if (t == 0) {
        RealState& s = st[b];
        if (ROW) {
            s.obj2 = v[0];
        } else {  // [obj, j] = min(objs): first minimiser, NaNs omitted as MATLAB's min (:354)
            int jm = 0;
            double best = sqrt(v[5]), o2 = v[5];
#pragma unroll
            for (int j = 1; j < RMAX; ++j) {
                const double o = sqrt(v[5 + j]);
                if (j < r && (o < best || (best != best && o == o))) { best = o; o2 = v[5 + j]; jm = j; }
            }
            s.obj2 = o2;
            s.objcol = jm;
        }
        s.nAX2 = v[1];
        s.nY2 = v[2];
        s.nJM2 = v[3];
        s.dY2 = v[4];
    }
}

__global__ __launch_bounds__(256) void finalize_r_kernel(int n, int m, int r, int nc, const double* optX,
                                                         const double* optY, const double* Xcur, const double* Ycur,
                                                         double* Xo, double* Yo, int32_t* iters, uint32_t* status,
                                                         double* muo, RealState* st, const double* Zb1,
                                                         const double* Zb2, const double* Yb1, const double* Yb2) {
    const int b = blockIdx.x;
    const bool have = st[b].opt_obj < INFINITY;
    const int os = st[b].optsrc;   // deferred opt_X copy (r = 1 wmode): the Z / Z2 buffer holds it
    const double* ox = (os == 1 && Zb1) ? Zb1 : ((os == 2 && Zb2) ? Zb2 : optX);
    const d2* sx = have ? reinterpret_cast<const d2*>(ox) + (long long)b * nc * n
                        : reinterpret_cast<const d2*>(Xcur) + (long long)b * r * n;
    const int oy = st[b].optysrc;   // deferred opt_Y copy (gyk_kernel): the Y[0] / Y[1] buffer holds it
    const double* oyp = (oy == 1 && Yb1) ? Yb1 : ((oy == 2 && Yb2) ? Yb2 : optY);
    const d2* sy = have ? reinterpret_cast<const d2*>(oyp) + (long long)b * nc * m
                        : reinterpret_cast<const d2*>(Ycur) + (long long)b * r * m;
    d2* dx = reinterpret_cast<d2*>(Xo) + (long long)b * nc * n;
    d2* dy = reinterpret_cast<d2*>(Yo) + (long long)b * nc * m;
    for (int k = threadIdx.x; k < nc * n; k += blockDim.x) dx[k] = sx[k];
    for (int i = threadIdx.x; i < nc * m; i += blockDim.x) dy[i] = sy[i];
    if (threadIdx.x == 0) {
        if (iters) iters[b] = st[b].iters;
        if (status) status[b] = (uint32_t)st[b].status | (have ? 0u : ACE_ST_NO_OPT);
        if (muo) muo[b] = st[b].mu;
    }
}

// ---------------------------------------------------------------- pipeline kernels
// A_norm = ||A||_F / sqrt(m) (tol guard :27-30) for one shared A; one work-group.
__global__ __launch_bounds__(1024) void anorm_kernel(long long count, int m, const double* A, double tol_abs,
                                                     double* anorm) {
    __shared__ double red[16];
    double s[1] = {0.0};
    for (long long k = threadIdx.x; k < count; k += blockDim.x) s[0] += A[k] * A[k];
    block_sum<1>(s, red);
    if (threadIdx.x == 0) {
        double a = sqrt(s[0]) / sqrt((double)m);
        anorm[0] = a < tol_abs ? 1.0 : a;
    }
}

// dst[i][:] = src[rows[i]][:] / anorm   (shared A: train / test row sets, :50-53)
__global__ __launch_bounds__(256) void gather_rows_kernel(int nrows, int n, const double* src, const int* rows,
                                                          const double* anorm, double* dst) {
    const int i = blockIdx.x;
    const double s = 1.0 / anorm[0];
    const d2* a = reinterpret_cast<const d2*>(src) + (long long)rows[i] * n;
    d2* d = reinterpret_cast<d2*>(dst) + (long long)i * n;
    for (int k = threadIdx.x; k < n; k += blockDim.x) d[k] = cscale(a[k], s);
}

// B_norm per realisation (:32-35) and Bn = B / B_norm
__global__ __launch_bounds__(256) void bnorm_kernel(int m, const double* B, double tol_abs, double* bnorm,
                                                    double* Bn) {
    const int b = blockIdx.x;
    __shared__ double red[16];
    const double* Bb = B + (long long)b * m;
    double s[1] = {0.0};
    for (int i = threadIdx.x; i < m; i += blockDim.x) s[0] += Bb[i] * Bb[i];
    block_sum<1>(s, red);
    double nb = sqrt(s[0]);
    if (nb < tol_abs) nb = 1.0;
    if (threadIdx.x == 0) bnorm[b] = nb;
    for (int i = threadIdx.x; i < m; i += blockDim.x) Bn[(long long)b * m + i] = Bb[i] / nb;
}

// per-realisation selection of B entries: dst[b][i] = src[b][rows[i]]
__global__ __launch_bounds__(256) void gather_b_kernel(int m, int nrows, const double* src, const int* rows,
                                                       double* dst) {
    const int b = blockIdx.x;
    for (int i = threadIdx.x; i < nrows; i += blockDim.x) dst[(long long)b * nrows + i] = src[(long long)b * m + rows[i]];
}

// dst[k][:] = src[idx[k]][:] (gather) or dst[idx[k]][:] = src[k][:] (scatter), len doubles
__global__ __launch_bounds__(256) void move_rows_kernel(long long len, const double* src, double* dst, const int* idx,
                                                        int scatter) {
    const int k = blockIdx.x;
    const long long so = (long long)(scatter ? k : idx[k]) * len, dof = (long long)(scatter ? idx[k] : k) * len;
    for (long long e = threadIdx.x; e < len; e += blockDim.x) dst[dof + e] = src[so + e];
}

// X <- X V with V the eigenvectors of X^H X in ascending eigenvalue order
// (inferLowRankV4_multi.m:263-264: [V, ~] = eig(X'*X); X = X*V -- MATLAB's eig of a
// Hermitian matrix returns ascending eigenvalues and it is not re-sorted).
__global__ __launch_bounds__(256) void gram_rotate_kernel(int n, int r, double* Xp, int* status) {
    const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    __shared__ d2 L0[ZT * ZHS];
    __shared__ d2 L1[ZT * ZHS];
    __shared__ double wv[ZT];
    __shared__ int asc[ZT];
    __shared__ JacobiShared jsh;
    d2* X = reinterpret_cast<d2*>(Xp) + (long long)b * r * n;
    const int nch = (n + ZT - 1) / ZT;
    auto stage_rows = [&](int c) {
        for (int e = t; e < ZT * ZT; e += 256) {
            const int i = e & 31, j = e >> 5, row = ZT * c + i;
            L0[i * ZHS + j] = (row < n && j < r) ? X[j * n + row] : make_double2(0.0, 0.0);
        }
    };
    d4v cr = {0.0, 0.0, 0.0, 0.0}, ci = {0.0, 0.0, 0.0, 0.0};
    for (int c = 0; c < nch; ++c) {
        stage_rows(c);
        __syncthreads();
        mm32_acc<true, false>(L0, L0, cr, ci, lane, w);  // X^H X
        __syncthreads();
    }
    store32(L0, cr, ci, lane, w);
    for (int e = t; e < ZT * ZT; e += 256) L1[(e >> 5) * ZHS + (e & 31)] = make_double2((e >> 5) == (e & 31), 0.0);
    __syncthreads();
    const int sz = r + (r & 1);
    if (jacobi_eig32(L0, L1, sz, wv, jsh) >= JAC_MAX_SWEEPS && t == 0 && status)
        atomicOr(&status[b], (int)ACE_ST_EIG_NOCONV);
    if (t < ZT) wv[t] = (t < r) ? wv[t] : INFINITY;  // the even-order pad sorts last
    __syncthreads();
    ascending_positions(wv, sz, asc);
    // L0[:, asc[c]] = V[:, c]  (columns in ascending eigenvalue order)
    for (int e = t; e < ZT * ZT; e += 256) {
        const int i = e >> 5, c = e & 31;
        const d2 q = L1[i * ZHS + c];
        if (c < sz) L0[i * ZHS + asc[c]] = q;
        else L0[i * ZHS + c] = make_double2(0.0, 0.0);
    }
    __syncthreads();
    for (int e = t; e < ZT * ZT; e += 256) L1[e / ZT * ZHS + e % ZT] = L0[e / ZT * ZHS + e % ZT];
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
        stage_rows(c);
        __syncthreads();
        mm32<false, false>(L0, L1, cr, ci, lane, w);  // X_c V
        __syncthreads();
        store32(L0, cr, ci, lane, w);
        __syncthreads();
        for (int e = t; e < ZT * ZT; e += 256) {
            const int i = e & 31, j = e >> 5, row = ZT * c + i;
            if (row < n && j < r) X[j * n + row] = L0[i * ZHS + j];
        }
        __syncthreads();
    }
}

// quality = 1 - norm(abs(A_test X) - B_test) / norm(B_test)   (:68), X = n x 1
__global__ __launch_bounds__(256) void quality_kernel(int n, int mte, const double* Ate, const double* Xp,
                                                      const double* Bte, double* q) {
    const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    __shared__ double red[16 * 2];
    __shared__ double part[4];
    const d2* X = reinterpret_cast<const d2*>(Xp) + (long long)b * n;
    const d2* A = reinterpret_cast<const d2*>(Ate);
    double v[2] = {0.0, 0.0};  // sum (|a_i x| - b_i)^2, sum b_i^2 (accumulated by thread 0)
    for (int i = 0; i < mte; ++i) {
        double re = 0.0, im = 0.0;
        for (int k = t; k < n; k += 256) {
            const d2 p = cmul(A[(long long)i * n + k], X[k]);
            re += p.x;
            im += p.y;
        }
        re = wave_sum(re);
        im = wave_sum(im);
        __syncthreads();
        if (lane == 0) { part[w] = re; red[w] = im; }
        __syncthreads();
        if (t == 0) {
            double sr = 0.0, si = 0.0;
            for (int k = 0; k < 4; ++k) { sr += part[k]; si += red[k]; }
            const double bi = Bte[(long long)b * mte + i];
            const double d = sqrt(sr * sr + si * si) - bi;
            v[0] += d * d;
            v[1] += bi * bi;
        }
    }
    if (t == 0) q[b] = 1.0 - sqrt(v[0]) / sqrt(v[1]);
}

// if max_quality < quality: X_max = X, Y_max = Y, max_quality = quality  (:79-83).
// On the first restart a NaN quality (B_test = 0) still seeds X_max, where the reference
// would fail on an undefined X_max.
__global__ __launch_bounds__(256) void keep_best_kernel(int n, int m, int first, const double* q, double* qmax,
                                                        const double* X, const double* Y, double* Xmax, double* Ymax) {
    const int b = blockIdx.x;
    const bool better = qmax[b] < q[b];
    if (!better && !(first && q[b] != q[b])) return;
    for (int k = threadIdx.x; k < 2 * n; k += blockDim.x) Xmax[(long long)b * 2 * n + k] = X[(long long)b * 2 * n + k];
    for (int i = threadIdx.x; i < 2 * m; i += blockDim.x) Ymax[(long long)b * 2 * m + i] = Y[(long long)b * 2 * m + i];
    if (threadIdx.x == 0 && better) qmax[b] = q[b];
}

// Refinement epilogue (:89-107): similarity rollback when the last restart's quality
// exceeds 0.6, then X, Y scaled by B_norm / A_norm.  Y_max has mt entries (train rows).
__global__ __launch_bounds__(256) void finish_kernel(int n, int m, int mt, const double* qlast, const double* Xr,
                                                     const double* Yr, const double* Xmax, const double* Ymax,
                                                     const double* anorm, const double* bnorm, double* Xo,
                                                     double* Yo, uint32_t* status) {
    const int b = blockIdx.x, t = threadIdx.x;
    __shared__ double red[16 * 4];
    __shared__ int roll;
    const d2* x = reinterpret_cast<const d2*>(Xr) + (long long)b * n;
    const d2* x0 = reinterpret_cast<const d2*>(Xmax) + (long long)b * n;
    double v[4] = {0.0, 0.0, 0.0, 0.0};  // Re, Im of X0^H X, ||X0||^2, ||X||^2
    for (int k = t; k < n; k += 256) {
        const d2 p = cmulc(x0[k], x[k]);
        v[0] += p.x;
        v[1] += p.y;
        v[2] += cabs2(x0[k]);
        v[3] += cabs2(x[k]);
    }
    block_sum<4>(v, red);
    if (t == 0) {
        int rb = 0;
        if (qlast[b] > 0.6) {
            const double sim = sqrt(v[0] * v[0] + v[1] * v[1]) / sqrt(v[2]) / sqrt(v[3]);
            rb = sim < 0.6;
        }
        roll = rb;
        if (rb && status) status[b] |= ACE_ST_ROLLBACK;
    }
    __syncthreads();
    const double s = bnorm[b] / anorm[0];
    d2* xo = reinterpret_cast<d2*>(Xo) + (long long)b * n;
    d2* yo = reinterpret_cast<d2*>(Yo) + (long long)b * m;
    const d2* ys = roll ? reinterpret_cast<const d2*>(Ymax) + (long long)b * mt
                        : reinterpret_cast<const d2*>(Yr) + (long long)b * m;
    const int ny = roll ? mt : m;
    for (int k = t; k < n; k += 256) xo[k] = cscale(roll ? x0[k] : x[k], s);
    for (int i = t; i < m; i += 256) yo[i] = i < ny ? cscale(ys[i], s) : make_double2(0.0, 0.0);
}
// dst[(idx ? idx[k] : k) * ld + col] = src[k] (or_mask == 0), else |= src[k] & or_mask
// (stage iteration counts, status bits)
__global__ __launch_bounds__(256) void put_col_kernel(int count, const int* src, const int* idx, int* dst, int ld,
                                                      int col, unsigned or_mask) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= count) return;
    const long long o = (long long)(idx ? idx[k] : k) * ld + col;
    dst[o] = or_mask ? (int)((unsigned)dst[o] | ((unsigned)src[k] & or_mask)) : src[k];
}

// the same for byte rows (partition tables)
__global__ __launch_bounds__(256) void move_bytes_kernel(long long len, const unsigned char* src, unsigned char* dst,
                                                         const int* idx, int scatter) {
    const int k = blockIdx.x;
    const long long so = (long long)(scatter ? k : idx[k]) * len, dof = (long long)(scatter ? idx[k] : k) * len;
    for (long long e = threadIdx.x; e < len; e += blockDim.x) dst[dof + e] = src[so + e];
}

__global__ __launch_bounds__(256) void flag_bits_kernel(int count, const unsigned char* flag, int* dst, unsigned bit) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < count && flag[k]) dst[k] = (int)((unsigned)dst[k] | bit);
}

__global__ __launch_bounds__(256) void fill_kernel(long long count, double v, double* dst) {
    const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < count) dst[k] = v;
}

// ---------------------------------------------------------------- per-realisation partitions (PartRows)
// G_ee^{-1}: gather the test-row block of G, invert it in LDS (Gauss-Jordan without pivoting: G_ee is a
// principal block of the HPD G = (I + K)^{-1}, eigenvalues in [1 / (1 + ||K||), 1])
__global__ __launch_bounds__(256) void part_geinv_kernel(PartRows pr, const double* Gp, double* geinvp, int* status) {
    const int b = blockIdx.x, t = threadIdx.x, m = pr.m, mt = pr.mt, te = m - mt;
    extern __shared__ d2 Hs[];   // te x te
    __shared__ int te_rows[PART_MAXTE];
    __shared__ int bad;
    const d2* G = reinterpret_cast<const d2*>(Gp);
    const int* rows = pr.rows + (long long)b * m;
    if (t < te) te_rows[t] = rows[mt + t];
    if (t == 0) bad = 0;
    __syncthreads();
    for (int e = t; e < te * te; e += 256) Hs[e] = G[(long long)te_rows[e / te] * m + te_rows[e % te]];
    __syncthreads();
    for (int k = 0; k < te; ++k) {   // in-place Gauss-Jordan inverse
        const d2 p = Hs[k * te + k];
        const double pr2 = cabs2(p);
        if (t == 0 && !(pr2 > 0.0)) bad = 1;
        const d2 pinv = make_double2(p.x / pr2, -p.y / pr2);
        __syncthreads();
        for (int e = t; e < te * te; e += 256) {   // H_ij -= H_ik H_kk^{-1} H_kj off the pivot row and column
            const int i = e / te, j = e % te;
            if (i == k || j == k) continue;
            Hs[e] = csub(Hs[e], cmul(cmul(Hs[i * te + k], pinv), Hs[k * te + j]));
        }
        __syncthreads();
        for (int e = t; e < te; e += 256) {        // then the pivot row (x H_kk^{-1}) and column (x -H_kk^{-1})
            if (e != k) {
                Hs[k * te + e] = cmul(pinv, Hs[k * te + e]);
                const d2 c = cmul(Hs[e * te + k], pinv);
                Hs[e * te + k] = make_double2(-c.x, -c.y);
            }
        }
        __syncthreads();
        if (t == 0) Hs[k * te + k] = pinv;
        __syncthreads();
    }
    d2* out = reinterpret_cast<d2*>(geinvp) + (long long)b * te * te;
    for (int e = t; e < te * te; e += 256) out[e] = Hs[e];
    if (t == 0 && bad && status) atomicOr(&status[b], (int)ACE_ST_EIG_NOCONV);
}

// g_t = u_t - G_te (G_ee^{-1} u_e), g_e = 0, with u = G T~ (whatever T~ holds on the test rows: its
// contributions cancel exactly in the Schur form).  The r columns go in chunks of GF_JC: each G_te entry
// is read once per chunk instead of once per column (r = 20: 3 reads instead of 20), with every output's
// products and their summation order (over the test rows, ascending) unchanged.
constexpr int GF_JC = 8;
__global__ __launch_bounds__(256) void part_gfix_kernel(int r, PartRows pr, const double* Gp, double* gp,
                                                        const RealState* rs) {
    const int b = blockIdx.x, t = threadIdx.x, m = pr.m, mt = pr.mt, te = m - mt;
    if (rs && rs[b].done) return;
    __shared__ d2 Ge[PART_MAXTE * PART_MAXTE / 4];   // G_ee^{-1} (te <= 48) or streamed from global
    __shared__ int te_rows[PART_MAXTE];
    __shared__ d2 ue[GF_JC][PART_MAXTE], de[GF_JC][PART_MAXTE];
    const d2* G = reinterpret_cast<const d2*>(Gp);
    const int* rows = pr.rows + (long long)b * m;
    const unsigned char* mask = pr.mask + (long long)b * pr.ldmask;
    const d2* gi = reinterpret_cast<const d2*>(pr.geinv) + (long long)b * te * te;
    const bool lds = te * te <= PART_MAXTE * PART_MAXTE / 4;
    if (t < te) te_rows[t] = rows[mt + t];
    if (lds)
        for (int e = t; e < te * te; e += 256) Ge[e] = gi[e];
    __syncthreads();
    d2* gb = reinterpret_cast<d2*>(gp) + (long long)b * r * m;
    for (int j0 = 0; j0 < r; j0 += GF_JC) {
        const int nj = min(GF_JC, r - j0);
        for (int e = t; e < nj * te; e += 256) {
            const int jj = e / te, f = e - jj * te;
            ue[jj][f] = gb[(long long)(j0 + jj) * m + te_rows[f]];
        }
        __syncthreads();
        for (int e = t; e < nj * te; e += 256) {   // d = G_ee^{-1} u_e per column
            const int jj = e / te, tt = e - jj * te;
            double re = 0.0, im = 0.0;
            for (int f = 0; f < te; ++f) {
                const d2 p = cmul(lds ? Ge[tt * te + f] : gi[tt * te + f], ue[jj][f]);
                re += p.x;
                im += p.y;
            }
            de[jj][tt] = make_double2(re, im);
        }
        __syncthreads();
        for (int i = t; i < m; i += 256) {
            if (!mask[i]) {
                for (int jj = 0; jj < nj; ++jj) gb[(long long)(j0 + jj) * m + i] = make_double2(0.0, 0.0);
                continue;
            }
            double re[GF_JC], im[GF_JC];
#pragma unroll
            for (int jj = 0; jj < GF_JC; ++jj) re[jj] = im[jj] = 0.0;
            for (int e = 0; e < te; ++e) {   // G[i][te_e] = conj(G[te_e][i]): row reads, coalesced over i
                const d2 gr = G[(long long)te_rows[e] * m + i], gc = make_double2(gr.x, -gr.y);
#pragma unroll
                for (int jj = 0; jj < GF_JC; ++jj) {
                    if (jj < nj) {
                        const d2 p = cmul(gc, de[jj][e]);
                        re[jj] += p.x;
                        im[jj] += p.y;
                    }
                }
            }
#pragma unroll
            for (int jj = 0; jj < GF_JC; ++jj)
                if (jj < nj) {
                    d2* g = gb + (long long)(j0 + jj) * m + i;
                    *g = csub(*g, make_double2(re[jj], im[jj]));
                }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void part_expand_kernel(int r, PartRows pr, const double* srcp, double* dstp) {
    const int b = blockIdx.y, j = blockIdx.x, m = pr.m, mt = pr.mt;
    const int* rows = pr.rows + (long long)b * m;
    const d2* src = reinterpret_cast<const d2*>(srcp) + ((long long)b * r + j) * mt;
    d2* dst = reinterpret_cast<d2*>(dstp) + ((long long)b * r + j) * m;
    for (int k = threadIdx.x; k < m; k += 256) dst[rows[k]] = k < mt ? src[k] : make_double2(0.0, 0.0);
}

__global__ __launch_bounds__(256) void part_compact_kernel(int r, PartRows pr, const double* srcp, double* dstp) {
    const int b = blockIdx.y, j = blockIdx.x, m = pr.m, mt = pr.mt;
    const int* rows = pr.rows + (long long)b * m;
    const d2* src = reinterpret_cast<const d2*>(srcp) + ((long long)b * r + j) * m;
    d2* dst = reinterpret_cast<d2*>(dstp) + ((long long)b * r + j) * mt;
    for (int k = threadIdx.x; k < mt; k += 256) dst[k] = src[rows[k]];
}

// quality_kernel on each realisation's own test rows (ascending, as setdiff returns them, :49)
__global__ __launch_bounds__(256) void part_quality_kernel(int n, PartRows pr, const double* Ap, const double* Xp,
                                                           const double* Bp, double* q) {
    const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6, m = pr.m, mt = pr.mt;
    __shared__ double red[16 * 2];
    __shared__ double part[4];
    const d2* X = reinterpret_cast<const d2*>(Xp) + (long long)b * n;
    const d2* A = reinterpret_cast<const d2*>(Ap);
    const int* rows = pr.rows + (long long)b * m;
    double v[2] = {0.0, 0.0};
    for (int i = mt; i < m; ++i) {
        const int row = rows[i];
        double re = 0.0, im = 0.0;
        for (int k = t; k < n; k += 256) {
            const d2 p = cmul(A[(long long)row * n + k], X[k]);
            re += p.x;
            im += p.y;
        }
        re = wave_sum(re);
        im = wave_sum(im);
        __syncthreads();
        if (lane == 0) { part[w] = re; red[w] = im; }
        __syncthreads();
        if (t == 0) {
            double sr = 0.0, si = 0.0;
            for (int k = 0; k < 4; ++k) { sr += part[k]; si += red[k]; }
            const double bi = Bp[(long long)b * m + row];
            const double d = sqrt(sr * sr + si * si) - bi;
            v[0] += d * d;
            v[1] += bi * bi;
        }
    }
    if (t == 0) q[b] = 1.0 - sqrt(v[0]) / sqrt(v[1]);
}
}  // namespace

void launch_init_r(int row_mode, int n, int m, int r, int batch, const double* X0, const double* P0, const double* B,
                   double* X, double* Y, double* M, double* N, RealState* rs, double mu0, hipStream_t st,
                   const PartRows* pr) {
    const unsigned char* mk = pr ? pr->mask : nullptr;
    const int ld = pr ? pr->ldmask : 0;
    if (row_mode)
        hipLaunchKernelGGL(init_r_kernel<true>, dim3(batch), dim3(256), 0, st, n, m, r, X0, P0, B, X, Y, M, N, rs, mu0,
                           mk, ld);
    else
        hipLaunchKernelGGL(init_r_kernel<false>, dim3(batch), dim3(256), 0, st, n, m, r, X0, P0, B, X, Y, M, N, rs,
                           mu0, mk, ld);
}
void launch_ystep_r(int row_mode, int m, int r, int batch, const double* S, const double* g, double* M,
                    const double* B, const double* Yold, double* Ynew, RealState* rs, hipStream_t st,
                    const PartRows* pr) {
    const unsigned char* mk = pr ? pr->mask : nullptr;
    const int ld = pr ? pr->ldmask : 0;
    if (row_mode)
        hipLaunchKernelGGL(ystep_r_kernel<true>, dim3(batch), dim3(256), 0, st, m, r, S, g, M, B, Yold, Ynew, rs, mk,
                           ld);
    else
        hipLaunchKernelGGL(ystep_r_kernel<false>, dim3(batch), dim3(256), 0, st, m, r, S, g, M, B, Yold, Ynew, rs, mk,
                           ld);
}
void launch_finalize_r(int n, int m, int r, int nc, int batch, const double* optX, const double* optY,
                       const double* Xc, const double* Yc, double* Xo, double* Yo, int32_t* iters, uint32_t* status,
                       double* mu, RealState* rs, hipStream_t st, const double* Zb1, const double* Zb2,
                       const double* Yb1, const double* Yb2) {
    hipLaunchKernelGGL(finalize_r_kernel, dim3(batch), dim3(256), 0, st, n, m, r, nc, optX, optY, Xc, Yc, Xo, Yo,
                       iters, status, mu, rs, Zb1, Zb2, Yb1, Yb2);
}

void launch_anorm(int m, int n, const double* A, double tol_abs, double* anorm, hipStream_t st) {
    hipLaunchKernelGGL(anorm_kernel, dim3(1), dim3(1024), 0, st, 2LL * m * n, m, A, tol_abs, anorm);
}
void launch_gather_rows(int nrows, int n, const double* src, const int* rows, const double* anorm, double* dst,
                        hipStream_t st) {
    if (nrows > 0) hipLaunchKernelGGL(gather_rows_kernel, dim3(nrows), dim3(256), 0, st, nrows, n, src, rows, anorm, dst);
}
void launch_bnorm(int m, int batch, const double* B, double tol_abs, double* bnorm, double* Bn, hipStream_t st) {
    hipLaunchKernelGGL(bnorm_kernel, dim3(batch), dim3(256), 0, st, m, B, tol_abs, bnorm, Bn);
}
void launch_gather_b(int m, int nrows, int batch, const double* src, const int* rows, double* dst, hipStream_t st) {
    if (nrows > 0) hipLaunchKernelGGL(gather_b_kernel, dim3(batch), dim3(256), 0, st, m, nrows, src, rows, dst);
}
void launch_move_rows(int count, long long len, const double* src, double* dst, const int* idx, bool scatter,
                      hipStream_t st) {
    if (count > 0)
        hipLaunchKernelGGL(move_rows_kernel, dim3(count), dim3(256), 0, st, len, src, dst, idx, scatter ? 1 : 0);
}
void launch_gram_rotate(int n, int r, int batch, double* X, int* status, hipStream_t st) {
    hipLaunchKernelGGL(gram_rotate_kernel, dim3(batch), dim3(256), 0, st, n, r, X, status);
}
void launch_quality(int n, int mte, int batch, const double* Ate, const double* X, const double* Bte, double* q,
                    hipStream_t st) {
    hipLaunchKernelGGL(quality_kernel, dim3(batch), dim3(256), 0, st, n, mte, Ate, X, Bte, q);
}
void launch_keep_best(int n, int m, int batch, bool first, const double* q, double* qmax, const double* X,
                      const double* Y, double* Xmax, double* Ymax, hipStream_t st) {
    hipLaunchKernelGGL(keep_best_kernel, dim3(batch), dim3(256), 0, st, n, m, first ? 1 : 0, q, qmax, X, Y, Xmax, Ymax);
}
void launch_finish(int n, int m, int mt, int batch, const double* qlast, const double* Xr, const double* Yr,
                   const double* Xmax, const double* Ymax, const double* anorm, const double* bnorm, double* Xo,
                   double* Yo, uint32_t* status, hipStream_t st) {
    hipLaunchKernelGGL(finish_kernel, dim3(batch), dim3(256), 0, st, n, m, mt, qlast, Xr, Yr, Xmax, Ymax, anorm, bnorm,
                       Xo, Yo, status);
}

void launch_put_col(int count, const int* src, const int* idx, int* dst, int ld, int col, unsigned or_mask,
                    hipStream_t st) {
    if (count > 0)
        hipLaunchKernelGGL(put_col_kernel, dim3((count + 255) / 256), dim3(256), 0, st, count, src, idx, dst, ld, col,
                           or_mask);
}
void launch_move_bytes(int count, long long len, const void* src, void* dst, const int* idx, bool scatter,
                       hipStream_t st) {
    if (count > 0)
        hipLaunchKernelGGL(move_bytes_kernel, dim3(count), dim3(256), 0, st, len, (const unsigned char*)src,
                           (unsigned char*)dst, idx, scatter ? 1 : 0);
}
void launch_flag_bits(int count, const unsigned char* flag, int* dst, unsigned bit, hipStream_t st) {
    if (count > 0) hipLaunchKernelGGL(flag_bits_kernel, dim3((count + 255) / 256), dim3(256), 0, st, count, flag, dst, bit);
}
void launch_part_geinv(int nb, const PartRows& pr, const double* G, double* geinv, int* status, hipStream_t st) {
    const int te = pr.m - pr.mt;
    if (nb > 0 && te > 0)
        hipLaunchKernelGGL(part_geinv_kernel, dim3(nb), dim3(256), (size_t)te * te * 16, st, pr, G, geinv, status);
}
void launch_part_gfix(int nb, int r, const PartRows& pr, const double* G, double* g, const RealState* rs,
                      hipStream_t st) {
    if (nb > 0) hipLaunchKernelGGL(part_gfix_kernel, dim3(nb), dim3(256), 0, st, r, pr, G, g, rs);
}
void launch_part_expand(int nb, int r, const PartRows& pr, const double* src, double* dst, hipStream_t st) {
    if (nb > 0) hipLaunchKernelGGL(part_expand_kernel, dim3(r, nb), dim3(256), 0, st, r, pr, src, dst);
}
void launch_part_compact(int nb, int r, const PartRows& pr, const double* src, double* dst, hipStream_t st) {
    if (nb > 0) hipLaunchKernelGGL(part_compact_kernel, dim3(r, nb), dim3(256), 0, st, r, pr, src, dst);
}
void launch_part_quality(int n, int nb, const PartRows& pr, const double* A, const double* X, const double* B,
                         double* q, hipStream_t st) {
    if (nb > 0) hipLaunchKernelGGL(part_quality_kernel, dim3(nb), dim3(256), 0, st, n, pr, A, X, B, q);
}
void launch_fill(long long count, double v, double* dst, hipStream_t st) {
    if (count > 0) hipLaunchKernelGGL(fill_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, count, v, dst);
}

}  // namespace ace
