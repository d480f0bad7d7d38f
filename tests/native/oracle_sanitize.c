/* Host ASan/UBSan exercise of the C restatement oracle (oracle/ace_oracle.c), SURVEY.md §5.
 * Built by `make -C oracle sanitize` into tests/native/oracle_sanitize; tests/test_sanitize.py
 * runs it.  Exit status non-zero on a sanitizer report or a failed check. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

int aceo_make_U(int m, int n, const double* A, double* U, int nthreads);
int aceo_infer_admm_r1(int variant, int use_rank_one, int fixed_iters, int m, int n, int tx, int rx, double mu0,
                       double rho, double tol_rel, double tol_abs, int maxiter, const double* A, const double* U,
                       const double* B, const double* X0, double* X, double* Y, int* iters, int* converged,
                       double* mu_out);
int aceo_infer_admm_r1_batch(int variant, int use_rank_one, int fixed_iters, int m, int n, int tx, int rx,
                             double mu0, double rho, double tol_rel, double tol_abs, int maxiter, int batch,
                             int a_shared, const double* A, const double* U, const double* B, const double* X0,
                             double* X, double* Y, int* iters, int* converged, double* mu_out, int nthreads);
int aceo_herm_eig(int n, const double* H, double* w, double* V);

static unsigned long long s = 88172645463325252ull;
static double uni(void) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    return (double)(s >> 11) / 9007199254740992.0;
}

int main(void) {
    const int tx = 4, rx = 4, n = 16, m = 40, batch = 3;
    double* A = malloc(sizeof(double) * 2 * m * n);
    double* U = malloc(sizeof(double) * 2 * n * n);
    double* B = malloc(sizeof(double) * batch * m);
    double* X0 = malloc(sizeof(double) * 2 * batch * n);
    double* X = malloc(sizeof(double) * 2 * batch * n);
    double* Y = malloc(sizeof(double) * 2 * batch * m);
    int it[3], cv[3];
    double mu[3];
    const double re[4] = {1, 0, -1, 0}, im[4] = {0, 1, 0, -1};
    for (int e = 0; e < m * n; ++e) {
        int k = (int)(uni() * 4) & 3;
        A[2 * e] = re[k] / 4.0;
        A[2 * e + 1] = im[k] / 4.0;
    }
    for (int i = 0; i < batch * m; ++i) B[i] = uni();
    B[5] = 0.0;   /* a zero magnitude (normalize_rows guard) */
    for (int i = 0; i < 2 * batch * n; ++i) X0[i] = uni() - 0.5;
    int fails = 0;
    fails += aceo_make_U(m, n, A, U, 2) != 0;
    for (int variant = 0; variant < 2; ++variant)
        for (int r1 = 0; r1 < 2; ++r1) {
            fails += aceo_infer_admm_r1(variant, r1, 0, m, n, tx, rx, 1e-3, 1.03, 1e-4, 1e-8, 60, A, U, B, X0, X, Y,
                                        it, cv, mu) != 0;
            fails += aceo_infer_admm_r1_batch(variant, r1, 1, m, n, tx, rx, 1e-3, 1.03, 1e-4, 1e-8, 30, batch, 1, A,
                                              U, B, X0, X, Y, it, cv, mu, 2) != 0;
            for (int i = 0; i < 2 * batch * n; ++i) fails += !isfinite(X[i]);
        }
    fails += aceo_infer_admm_r1(0, 0, 0, m, 15, tx, rx, 1e-3, 1.03, 1e-4, 1e-8, 60, A, U, B, X0, X, Y, it, cv, mu) !=
             -2;   /* n != tx * rx */
    double H[2 * 16 * 16], w[16], V[2 * 16 * 16];
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j <= i; ++j) {
            double a = uni() - 0.5, b = i == j ? 0.0 : uni() - 0.5;
            H[2 * (i * 16 + j)] = a; H[2 * (i * 16 + j) + 1] = b;
            H[2 * (j * 16 + i)] = a; H[2 * (j * 16 + i) + 1] = -b;
        }
    fails += aceo_herm_eig(16, H, w, V) != 0;
    for (int i = 1; i < 16; ++i) fails += w[i] < w[i - 1];
    free(A); free(U); free(B); free(X0); free(X); free(Y);
    if (fails) { fprintf(stderr, "%d checks failed\n", fails); return 1; }
    printf("OK\n");
    return 0;
}
