/*
 * CPU oracle (plain C, fp64) for the 2ACE ADMM refinement solve.
 *
 * TEST INFRASTRUCTURE ONLY: linked/loaded only by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg, and there only as the checker / the CPU
 * baseline ("port").  The product path never calls it.
 *
 * Parity status: **parity unpinned against MATLAB** (no MATLAB/Octave in the
 * image, no reference ADMM outputs exist).  This file is an
 * independent second restatement of the MATLAB code, cross-checked against the
 * numpy restatement oracle/ace_oracle.py in tests/test_oracle.py.
 *
 * It follows main/src/my_recovery_algorithms/ADMM_v2/inferLowRankV4_multi.m
 * (reference root /root/reference):
 *   InferADMM :281-386   (loop :318-383)       -> aceo_infer_admm_r1
 *   ArgMinX   :401-409   (lambda = 0 branch)
 *   ArgMinZ   :423-485   (eig(E*E') :428, profile :437-464, rescale :469-484)
 *   ArgMinY   :511-533,  normalize_rows :538-559
 *   U = inv(A'*A + I) :242 / :288            -> aceo_make_U (Gauss-Jordan)
 * and inferLowRank_Nuclear.m:411-439 for the nuclear Z-step (r = 1: the SVD
 * soft threshold of an n-by-1 iterate is a norm shrink).
 *
 * Scope: r = 1 (the refinement stage, the benchmark unit of SURVEY.md §8d).
 * At r = 1 the row-wise and column-wise modes of InferADMM coincide.
 *
 * Complex numbers are interleaved (re, im) doubles; matrices row-major.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define VAR_A2ONLY 0
#define VAR_NUCLEAR 1

/* ---------------------------------------------------------------- helpers */
static double nrm2c(const double* x, int n) { /* ||x||_2, complex, sequential */
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += x[2 * i] * x[2 * i] + x[2 * i + 1] * x[2 * i + 1];
    return sqrt(s);
}
static double nrm2c_diff(const double* x, const double* y, int n) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) {
        double a = x[2 * i] - y[2 * i], b = x[2 * i + 1] - y[2 * i + 1];
        s += a * a + b * b;
    }
    return sqrt(s);
}

/* y = L x, L rows x cols complex row-major; 4 partial accumulators per output */
static void matvec(const double* L, int rows, int cols, const double* x, double* y) {
    for (int i = 0; i < rows; ++i) {
        const double* a = L + (size_t)2 * i * cols;
        double r0 = 0, r1 = 0, i0 = 0, i1 = 0;
        int k = 0;
        for (; k + 1 < cols; k += 2) {
            double ar = a[2 * k], ai = a[2 * k + 1], br = a[2 * k + 2], bi = a[2 * k + 3];
            double xr = x[2 * k], xi = x[2 * k + 1], yr = x[2 * k + 2], yi = x[2 * k + 3];
            r0 += ar * xr - ai * xi;
            i0 += ar * xi + ai * xr;
            r1 += br * yr - bi * yi;
            i1 += br * yi + bi * yr;
        }
        for (; k < cols; ++k) {
            double ar = a[2 * k], ai = a[2 * k + 1], xr = x[2 * k], xi = x[2 * k + 1];
            r0 += ar * xr - ai * xi;
            i0 += ar * xi + ai * xr;
        }
        y[2 * i] = r0 + r1;
        y[2 * i + 1] = i0 + i1;
    }
}

/* y = L^H x, L rows x cols, y has cols entries */
static void matvec_h(const double* L, int rows, int cols, const double* x, double* y) {
    memset(y, 0, sizeof(double) * 2 * cols);
    for (int i = 0; i < rows; ++i) {
        const double* a = L + (size_t)2 * i * cols;
        double xr = x[2 * i], xi = x[2 * i + 1];
        for (int k = 0; k < cols; ++k) {
            double ar = a[2 * k], ai = a[2 * k + 1];
            y[2 * k] += ar * xr + ai * xi;      /* conj(a) * x */
            y[2 * k + 1] += ar * xi - ai * xr;
        }
    }
}

/* ------------------------------------------------ Hermitian Jacobi eigen */
/* Cyclic Jacobi on an n x n Hermitian matrix H (destroyed).  Eigenvalues in w
 * (unsorted), eigenvectors in columns of V (row-major n x n complex). */
static void herm_jacobi(int n, double* H, double* w, double* V) {
    memset(V, 0, sizeof(double) * 2 * n * n);
    for (int i = 0; i < n; ++i) V[2 * (i * n + i)] = 1.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        int rotated = 0;
        for (int p = 0; p < n - 1; ++p)
            for (int q = p + 1; q < n; ++q) {
                double a = H[2 * (p * n + p)], b = H[2 * (q * n + q)];
                double cr = H[2 * (p * n + q)], ci = H[2 * (p * n + q) + 1];
                double ac = hypot(cr, ci);
                if (ac == 0.0 || ac <= 1e-300) continue;
                if (ac * ac <= 1e-32 * fabs(a * b)) continue; /* converged pair */
                rotated = 1;
                double er = cr / ac, ei = ci / ac; /* e^{i phi} */
                double zeta = (b - a) / (2.0 * ac);
                double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                double cs = 1.0 / sqrt(1.0 + t * t), sn = t * cs;
                /* J = [[cs, sn], [-sn e^{-i phi}, cs e^{-i phi}]]; H <- J^H H J, V <- V J */
                /* columns: H[:,p], H[:,q] */
                for (int k = 0; k < n; ++k) {
                    double hpr = H[2 * (k * n + p)], hpi = H[2 * (k * n + p) + 1];
                    double hqr = H[2 * (k * n + q)], hqi = H[2 * (k * n + q) + 1];
                    /* hq * e^{-i phi} */
                    double qr = hqr * er + hqi * ei, qi = hqi * er - hqr * ei;
                    H[2 * (k * n + p)] = cs * hpr - sn * qr;
                    H[2 * (k * n + p) + 1] = cs * hpi - sn * qi;
                    H[2 * (k * n + q)] = sn * hpr + cs * qr;
                    H[2 * (k * n + q) + 1] = sn * hpi + cs * qi;
                    double vpr = V[2 * (k * n + p)], vpi = V[2 * (k * n + p) + 1];
                    double vqr = V[2 * (k * n + q)], vqi = V[2 * (k * n + q) + 1];
                    double wr = vqr * er + vqi * ei, wi = vqi * er - vqr * ei;
                    V[2 * (k * n + p)] = cs * vpr - sn * wr;
                    V[2 * (k * n + p) + 1] = cs * vpi - sn * wi;
                    V[2 * (k * n + q)] = sn * vpr + cs * wr;
                    V[2 * (k * n + q) + 1] = sn * vpi + cs * wi;
                }
                /* rows: conj(J)^T applied: H[p,:], H[q,:] */
                for (int k = 0; k < n; ++k) {
                    double hpr = H[2 * (p * n + k)], hpi = H[2 * (p * n + k) + 1];
                    double hqr = H[2 * (q * n + k)], hqi = H[2 * (q * n + k) + 1];
                    /* hq * e^{+i phi} */
                    double qr = hqr * er - hqi * ei, qi = hqi * er + hqr * ei;
                    H[2 * (p * n + k)] = cs * hpr - sn * qr;
                    H[2 * (p * n + k) + 1] = cs * hpi - sn * qi;
                    H[2 * (q * n + k)] = sn * hpr + cs * qr;
                    H[2 * (q * n + k) + 1] = sn * hpi + cs * qi;
                }
                H[2 * (p * n + q)] = H[2 * (p * n + q) + 1] = 0.0;
                H[2 * (q * n + p)] = H[2 * (q * n + p) + 1] = 0.0;
                H[2 * (p * n + p) + 1] = H[2 * (q * n + q) + 1] = 0.0;
            }
        if (!rotated) break;
    }
    for (int i = 0; i < n; ++i) w[i] = H[2 * (i * n + i)];
}

/* --------------------------------------------------------------- ArgMinZ */
static int ceil_i(double x) { return (int)ceil(x); }

/* inferLowRankV4_multi.m:437-464 */
static int rank_profile(int tx, int rx, int m, int n, int use_rank_one, int* rl, double* fl) {
    int sz = tx < rx ? tx : rx;
    int r0 = ceil_i(sqrt((double)sz) * 0.5), r1 = ceil_i(sqrt((double)sz) * 0.7);
    int r2 = ceil_i(sqrt((double)sz)), r3 = ceil_i(sqrt((double)sz) * 2.0);
    if (r3 > sz) r3 = sz;
    if (use_rank_one) { rl[0] = 1; fl[0] = 0.95; return 1; }
    if (m >= n * 3) { rl[0] = r3; fl[0] = 0.995; return 1; }
    if (r1 <= 2) { rl[0] = r2; fl[0] = 0.95; return 1; }
    if (r0 <= 2) { rl[0] = r1; rl[1] = r2; rl[2] = r3; fl[0] = 0.9; fl[1] = 0.95; fl[2] = 0.995; return 3; }
    rl[0] = r0; rl[1] = r1; rl[2] = r2; rl[3] = r3;
    fl[0] = 0.8; fl[1] = 0.9; fl[2] = 0.95; fl[3] = 0.995;
    return 4;
}

typedef struct {
    int tx, rx;
    double *E, *H, *V, *w, *tmp;
    int *order;
} zwork;

/* Z = ArgMinZ(X, N, mu) for r = 1 (E is tx x rx, column-major reshape of z) */
static void argmin_z_lowrank(zwork* zw, const double* X, const double* N, double mu, int m, int n,
                             int use_rank_one, double* Z) {
    int tx = zw->tx, rx = zw->rx;
    double* E = zw->E; /* row-major tx x rx: E[i][j] = z[i + tx*j] */
    for (int j = 0; j < rx; ++j)
        for (int i = 0; i < tx; ++i) {
            int k = i + tx * j;
            E[2 * (i * rx + j)] = X[2 * k] + N[2 * k] / mu;
            E[2 * (i * rx + j) + 1] = X[2 * k + 1] + N[2 * k + 1] / mu;
        }
    double* H = zw->H; /* H = E E^H, tx x tx */
    for (int i = 0; i < tx; ++i)
        for (int j = i; j < tx; ++j) {
            double sr = 0, si = 0;
            for (int k = 0; k < rx; ++k) {
                double ar = E[2 * (i * rx + k)], ai = E[2 * (i * rx + k) + 1];
                double br = E[2 * (j * rx + k)], bi = E[2 * (j * rx + k) + 1];
                sr += ar * br + ai * bi;
                si += ai * br - ar * bi;
            }
            H[2 * (i * tx + j)] = sr;
            H[2 * (i * tx + j) + 1] = si;
            H[2 * (j * tx + i)] = sr;
            H[2 * (j * tx + i) + 1] = -si;
        }
    for (int i = 0; i < tx; ++i) H[2 * (i * tx + i) + 1] = 0.0;
    herm_jacobi(tx, H, zw->w, zw->V);
    /* emulate LAPACK's ascending order, then MATLAB's stable descending sort (:429-430) */
    int* asc = zw->order;
    for (int i = 0; i < tx; ++i) asc[i] = i;
    for (int i = 1; i < tx; ++i) { /* stable insertion sort ascending by w */
        int v = asc[i], j = i - 1;
        while (j >= 0 && zw->w[asc[j]] > zw->w[v]) { asc[j + 1] = asc[j]; --j; }
        asc[j + 1] = v;
    }
    double s2a[64], s2[64], scl[64];
    int idx[64];
    for (int i = 0; i < tx; ++i) s2a[i] = fmax(0.0, zw->w[asc[i]]);
    for (int i = 0; i < tx; ++i) idx[i] = i;
    for (int i = 1; i < tx; ++i) { /* stable sort descending on s2a */
        int v = idx[i], j = i - 1;
        while (j >= 0 && s2a[idx[j]] < s2a[v]) { idx[j + 1] = idx[j]; --j; }
        idx[j + 1] = v;
    }
    for (int i = 0; i < tx; ++i) { s2[i] = s2a[idx[i]]; scl[i] = 1.0; }
    int rl[4];
    double fl[4];
    int np = rank_profile(tx, rx, m, n, use_rank_one, rl, fl);
    int any = 0;
    for (int p = 0; p < np; ++p) { /* :470-480 */
        int r = rl[p];
        double f = fl[p], vr = 0.0, v = 0.0;
        for (int i = 0; i < r; ++i) vr += s2[i];
        for (int i = 0; i < tx; ++i) v += s2[i];
        if (vr < v * f) {
            double scale = vr / (v - vr) * (1.0 / f - 1.0);
            if (scale > 1.0) scale = 1.0;
            for (int i = r; i < tx; ++i) { s2[i] *= scale; scl[idx[i]] *= scale; }
        }
    }
    for (int i = 0; i < tx; ++i) any |= scl[i] < 1.0;
    if (!any) {
        for (int k = 0; k < n; ++k) {
            Z[2 * k] = X[2 * k] + N[2 * k] / mu;
            Z[2 * k + 1] = X[2 * k + 1] + N[2 * k + 1] / mu;
        }
        return;
    }
    /* Z = U diag(sqrt(scl)) U^H E; U column c = eigenvector asc[c] */
    double* T = zw->tmp; /* T = diag(sqrt) U^H E  (tx x rx) */
    for (int c = 0; c < tx; ++c) {
        double ws = sqrt(scl[c]);
        int col = asc[c];
        for (int j = 0; j < rx; ++j) {
            double sr = 0, si = 0;
            for (int i = 0; i < tx; ++i) {
                double ur = zw->V[2 * (i * tx + col)], ui = zw->V[2 * (i * tx + col) + 1];
                double er = E[2 * (i * rx + j)], ei = E[2 * (i * rx + j) + 1];
                sr += ur * er + ui * ei;
                si += ur * ei - ui * er;
            }
            T[2 * (c * rx + j)] = ws * sr;
            T[2 * (c * rx + j) + 1] = ws * si;
        }
    }
    for (int i = 0; i < tx; ++i)
        for (int j = 0; j < rx; ++j) {
            double sr = 0, si = 0;
            for (int c = 0; c < tx; ++c) {
                int col = asc[c];
                double ur = zw->V[2 * (i * tx + col)], ui = zw->V[2 * (i * tx + col) + 1];
                double tr = T[2 * (c * rx + j)], ti = T[2 * (c * rx + j) + 1];
                sr += ur * tr - ui * ti;
                si += ur * ti + ui * tr;
            }
            int k = i + tx * j;
            Z[2 * k] = sr;
            Z[2 * k + 1] = si;
        }
}

/* inferLowRank_Nuclear.m:411-439 at r = 1 */
static void argmin_z_nuclear(const double* X, const double* N, double mu, int n, double* Z) {
    double s = 0.0;
    for (int k = 0; k < n; ++k) {
        double a = X[2 * k] + N[2 * k] / mu, b = X[2 * k + 1] + N[2 * k + 1] / mu;
        Z[2 * k] = a;
        Z[2 * k + 1] = b;
        s += a * a + b * b;
    }
    double nz = sqrt(s);
    double f = nz > 0 ? fmax(0.0, nz - 1.0 / mu) / nz : 0.0;
    for (int k = 0; k < 2 * n; ++k) Z[k] *= f;
}

/* ------------------------------------------------------------ U = inv() */
typedef struct {
    int n, m, nth, tid;
    const double* A;
    double* W; /* n x 2n augmented not used: in-place Gauss-Jordan on U */
    pthread_barrier_t* bar;
} gj_arg;

static void* gj_worker(void* p) {
    gj_arg* g = (gj_arg*)p;
    int n = g->n, m = g->m, nth = g->nth, tid = g->tid;
    double* U = g->W;
    const double* A = g->A;
    /* U = A^H A + I, rows split over threads */
    for (int i = tid; i < n; i += nth)
        for (int j = 0; j < n; ++j) {
            double sr = (i == j) ? 1.0 : 0.0, si = 0.0;
            for (int k = 0; k < m; ++k) {
                double ar = A[2 * ((size_t)k * n + i)], ai = A[2 * ((size_t)k * n + i) + 1];
                double br = A[2 * ((size_t)k * n + j)], bi = A[2 * ((size_t)k * n + j) + 1];
                sr += ar * br + ai * bi;
                si += ar * bi - ai * br;
            }
            U[2 * ((size_t)i * n + j)] = sr;
            U[2 * ((size_t)i * n + j) + 1] = si;
        }
    pthread_barrier_wait(g->bar);
    /* in-place Gauss-Jordan inverse (HPD, no pivoting) */
    double* rowk = (double*)malloc(sizeof(double) * 2 * n);
    for (int k = 0; k < n; ++k) {
        /* every thread reads pivot row k (after the barrier it is final) */
        double pr = U[2 * ((size_t)k * n + k)], pi = U[2 * ((size_t)k * n + k) + 1];
        double den = pr * pr + pi * pi, ir = pr / den, ii = -pi / den; /* 1/pivot */
        for (int j = 0; j < n; ++j) {
            double ar = (j == k) ? 1.0 : U[2 * ((size_t)k * n + j)];
            double ai = (j == k) ? 0.0 : U[2 * ((size_t)k * n + j) + 1];
            rowk[2 * j] = ar * ir - ai * ii;
            rowk[2 * j + 1] = ar * ii + ai * ir;
        }
        pthread_barrier_wait(g->bar);
        for (int i = tid; i < n; i += nth) {
            double* ui = U + 2 * (size_t)i * n;
            if (i == k) {
                memcpy(ui, rowk, sizeof(double) * 2 * n);
                continue;
            }
            double fr = ui[2 * k], fi = ui[2 * k + 1];
            ui[2 * k] = 0.0;
            ui[2 * k + 1] = 0.0;
            for (int j = 0; j < n; ++j) {
                double ar = rowk[2 * j], ai = rowk[2 * j + 1];
                ui[2 * j] -= fr * ar - fi * ai;
                ui[2 * j + 1] -= fr * ai + fi * ar;
            }
        }
        pthread_barrier_wait(g->bar);
    }
    free(rowk);
    return NULL;
}

/* U = inv(A^H A + I), A m x n (inferLowRankV4_multi.m:242 / :288) */
int aceo_make_U(int m, int n, const double* A, double* U, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    pthread_t th[256];
    gj_arg args[256];
    if (nthreads > 256) nthreads = 256;
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
    for (int t = 0; t < nthreads; ++t) {
        args[t] = (gj_arg){n, m, nthreads, t, A, U, &bar};
        if (t) pthread_create(&th[t], NULL, gj_worker, &args[t]);
    }
    gj_worker(&args[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    pthread_barrier_destroy(&bar);
    return 0;
}

/* --------------------------------------------------------------- InferADMM */
typedef struct {
    int variant, use_rank_one, fixed_iters, m, n, tx, rx, maxiter;
    double mu0, rho, tol_rel, tol_abs;
} aceo_cfg;

/* InferADMM at r = 1 (inferLowRankV4_multi.m:281-386).  U must be
 * inv(A'A + I).  Outputs opt_X (n) and opt_Y (m). */
static int infer_admm_r1(const aceo_cfg* c, const double* A, const double* U, const double* B,
                         const double* X0, double* Xo, double* Yo, int* iters_o, int* conv_o,
                         double* mu_o) {
    int m = c->m, n = c->n;
    size_t nb = sizeof(double) * 2 * n, mb = sizeof(double) * 2 * m;
    double* buf = (double*)calloc((size_t)2 * (9 * n + 9 * m) + 64 * c->tx * (c->tx + c->rx) + 64, sizeof(double));
    if (!buf) return -1;
    double *X = buf, *Z = X + 2 * n, *Z0 = Z + 2 * n, *N = Z0 + 2 * n, *W = N + 2 * n, *V = W + 2 * n,
           *optX = V + 2 * n, *AtY = optX + 2 * n, *AtY0 = AtY + 2 * n;
    double *AX = AtY0 + 2 * n, *Y = AX + 2 * m, *Y0 = Y + 2 * m, *M = Y0 + 2 * m, *S = M + 2 * m,
           *optY = S + 2 * m, *JM = optY + 2 * m;
    zwork zw;
    zw.tx = c->tx;
    zw.rx = c->rx;
    zw.E = JM + 2 * m;
    zw.H = zw.E + 2 * c->tx * c->rx;
    zw.V = zw.H + 2 * c->tx * c->tx;
    zw.tmp = zw.V + 2 * c->tx * c->tx;
    zw.w = zw.tmp + 2 * c->tx * c->rx;
    int order[64];
    zw.order = order;

    memcpy(X, X0, nb);
    matvec(A, m, n, X, AX);                                     /* :299 */
    double nB = 0;
    for (int i = 0; i < m; ++i) nB += B[i] * B[i];
    nB = sqrt(nB);
    double sc = nB / nrm2c(AX, m);                              /* :301 */
    for (int k = 0; k < 2 * n; ++k) X[k] *= sc;
    matvec(A, m, n, X, AX);                                     /* :307 */
    for (int i = 0; i < m; ++i) {                               /* :308 normalize_rows */
        double d = hypot(AX[2 * i], AX[2 * i + 1]);
        double yr = AX[2 * i], yi = AX[2 * i + 1];
        if (d == 0) { yr = 1.0; yi = 0.0; d = 1.0; }
        Y[2 * i] = yr * (B[i] / d);
        Y[2 * i + 1] = yi * (B[i] / d);
    }
    memset(N, 0, nb);
    memset(M, 0, mb);
    if (c->variant == VAR_NUCLEAR) argmin_z_nuclear(X, N, 1.0, n, Z);  /* :309 */
    else argmin_z_lowrank(&zw, X, N, 1.0, m, n, c->use_rank_one, Z);
    matvec_h(A, m, n, Y, AtY);                                  /* :310 */

    double mu = c->mu0, opt_obj = INFINITY, last_res = INFINITY;
    int have_opt = 0, converged = 0, it;
    for (it = 1; it <= c->maxiter; ++it) {
        memcpy(Y0, Y, mb);
        memcpy(Z0, Z, nb);
        memcpy(AtY0, AtY, nb);
        /* ArgMinX :404: X = U (A'(Y - M/mu) + Z - N/mu) */
        for (int i = 0; i < 2 * m; ++i) S[i] = Y[i] - M[i] / mu;
        matvec_h(A, m, n, S, W);
        for (int k = 0; k < 2 * n; ++k) V[k] = W[k] + Z[k] - N[k] / mu;
        matvec(U, n, n, V, X);
        matvec(A, m, n, X, AX);                                 /* :326 */
        for (int i = 0; i < m; ++i) {                           /* ArgMinY :511-522 */
            double yr = AX[2 * i] + M[2 * i] / mu, yi = AX[2 * i + 1] + M[2 * i + 1] / mu;
            double d = sqrt(yr * yr + yi * yi);
            if (d == 0) { yr = 1.0; yi = 0.0; d = 1.0; }
            double f = (B[i] / d + mu) / (1 + mu);
            Y[2 * i] = yr * f;
            Y[2 * i + 1] = yi * f;
        }
        matvec_h(A, m, n, Y, AtY);                              /* :330 */
        if (c->variant == VAR_NUCLEAR) argmin_z_nuclear(X, N, mu, n, Z);   /* :333 */
        else argmin_z_lowrank(&zw, X, N, mu, m, n, c->use_rank_one, Z);
        double jm2 = 0, jn2 = 0;
        for (int i = 0; i < 2 * m; ++i) { JM[i] = AX[i] - Y[i]; M[i] += mu * JM[i]; jm2 += JM[i] * JM[i]; }
        for (int k = 0; k < 2 * n; ++k) { double d = X[k] - Z[k]; N[k] += mu * d; jn2 += d * d; }
        double obj = 0;                                         /* :345 */
        for (int i = 0; i < m; ++i) {
            double d = sqrt(AX[2 * i] * AX[2 * i] + AX[2 * i + 1] * AX[2 * i + 1]) - B[i];
            obj += d * d;
        }
        obj = sqrt(obj);
        if (obj < opt_obj) {
            opt_obj = obj;
            memcpy(optX, X, nb);
            memcpy(optY, Y, mb);
            have_opt = 1;
        }
        double nAX = nrm2c(AX, m), nY = nrm2c(Y, m), nX = nrm2c(X, n), nZ = nrm2c(Z, n);
        double dZ = nrm2c_diff(Z, Z0, n), dY = nrm2c_diff(Y, Y0, m), dAtY = nrm2c_diff(AtY, AtY0, n);
        double nAtY = nrm2c(AtY, n);
        double res_prim = sqrt(jm2 + jn2);                      /* :364-366 */
        double res_dual = mu * sqrt(dAtY * dAtY + dZ * dZ);
        double res_comb = sqrt(res_prim * res_prim + dY * dY + dZ * dZ);
        double mx1 = fmax(nAX, nY), mx2 = fmax(nX, nZ);
        double t_prim = c->tol_abs * sqrt((double)(m + n)) + c->tol_rel * sqrt(mx1 * mx1 + mx2 * mx2);
        double t_dual = c->tol_abs * sqrt((double)n * 2) + c->tol_rel * sqrt(nAtY * nAtY + nZ * nZ);
        double t_comb = c->tol_abs * sqrt((double)(m + n) * 2) +
                        c->tol_rel * sqrt(mx1 * mx1 + mx2 * mx2 + nY * nY + nZ * nZ);
        if ((res_prim < t_prim && res_dual < t_dual) || res_comb < t_comb) {   /* :372 */
            converged = 1;
            if (!c->fixed_iters) break;
        }
        if (res_comb > last_res * 0.9) mu *= c->rho;           /* :379-381 */
        last_res = res_comb;
    }
    if (it > c->maxiter) it = c->maxiter;
    if (!have_opt) { memcpy(optX, X, nb); memcpy(optY, Y, mb); }
    memcpy(Xo, optX, nb);
    memcpy(Yo, optY, mb);
    if (iters_o) *iters_o = it;
    if (conv_o) *conv_o = converged;
    if (mu_o) *mu_o = mu;
    free(buf);
    return 0;
}

int aceo_infer_admm_r1(int variant, int use_rank_one, int fixed_iters, int m, int n, int tx, int rx,
                       double mu0, double rho, double tol_rel, double tol_abs, int maxiter,
                       const double* A, const double* U, const double* B, const double* X0,
                       double* X, double* Y, int* iters, int* converged, double* mu_out) {
    if (tx * rx != n || tx > 64 || rx > 64) return -2;
    aceo_cfg c = {variant, use_rank_one, fixed_iters, m, n, tx, rx, maxiter, mu0, rho, tol_rel, tol_abs};
    return infer_admm_r1(&c, A, U, B, X0, X, Y, iters, converged, mu_out);
}

/* ------------------------------------------------------ batched, threaded */
typedef struct {
    const aceo_cfg* c;
    int a_shared, batch, tid, nth;
    const double *A, *U, *B, *X0;
    double *X, *Y;
    int *iters, *conv;
    double* mu;
    int rc;
} batch_arg;

static void* batch_worker(void* p) {
    batch_arg* a = (batch_arg*)p;
    const aceo_cfg* c = a->c;
    size_t an = (size_t)2 * c->m * c->n, un = (size_t)2 * c->n * c->n;
    for (int b = a->tid; b < a->batch; b += a->nth) {
        const double* Ab = a->A + (a->a_shared ? 0 : b * an);
        const double* Ub = a->U + (a->a_shared ? 0 : b * un);
        int rc = infer_admm_r1(c, Ab, Ub, a->B + (size_t)b * c->m, a->X0 + (size_t)2 * b * c->n,
                               a->X + (size_t)2 * b * c->n, a->Y + (size_t)2 * b * c->m,
                               a->iters + b, a->conv + b, a->mu + b);
        if (rc) a->rc = rc;
    }
    return NULL;
}

/* Batch of independent refinement solves, one realisation per thread at a time.
 * A/U are shared (a_shared=1) or per-realisation.  U must be precomputed. */
int aceo_infer_admm_r1_batch(int variant, int use_rank_one, int fixed_iters, int m, int n, int tx, int rx,
                             double mu0, double rho, double tol_rel, double tol_abs, int maxiter,
                             int batch, int a_shared, const double* A, const double* U, const double* B,
                             const double* X0, double* X, double* Y, int* iters, int* converged,
                             double* mu_out, int nthreads) {
    if (tx * rx != n || tx > 64 || rx > 64) return -2;
    aceo_cfg c = {variant, use_rank_one, fixed_iters, m, n, tx, rx, maxiter, mu0, rho, tol_rel, tol_abs};
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    batch_arg args[256];
    for (int t = 0; t < nthreads; ++t) {
        args[t] = (batch_arg){&c, a_shared, batch, t, nthreads, A, U, B, X0, X, Y, iters, converged, mu_out, 0};
        if (t) pthread_create(&th[t], NULL, batch_worker, &args[t]);
    }
    batch_worker(&args[0]);
    int rc = args[0].rc;
    for (int t = 1; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        if (args[t].rc) rc = args[t].rc;
    }
    return rc;
}

/* Hermitian eigen-decomposition exposed for tests (Jacobi): w ascending. */
int aceo_herm_eig(int n, const double* H, double* w, double* V) {
    double* Hc = (double*)malloc(sizeof(double) * 2 * n * n);
    double* Vt = (double*)malloc(sizeof(double) * 2 * n * n);
    double* wt = (double*)malloc(sizeof(double) * n);
    int* o = (int*)malloc(sizeof(int) * n);
    memcpy(Hc, H, sizeof(double) * 2 * n * n);
    herm_jacobi(n, Hc, wt, Vt);
    for (int i = 0; i < n; ++i) o[i] = i;
    for (int i = 1; i < n; ++i) {
        int v = o[i], j = i - 1;
        while (j >= 0 && wt[o[j]] > wt[v]) { o[j + 1] = o[j]; --j; }
        o[j + 1] = v;
    }
    for (int c = 0; c < n; ++c) {
        w[c] = wt[o[c]];
        for (int i = 0; i < n; ++i) {
            V[2 * (i * n + c)] = Vt[2 * (i * n + o[c])];
            V[2 * (i * n + c) + 1] = Vt[2 * (i * n + o[c]) + 1];
        }
    }
    free(Hc); free(Vt); free(wt); free(o);
    return 0;
}
