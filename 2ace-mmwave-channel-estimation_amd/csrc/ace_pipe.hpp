// Launchers of the recovery-pipeline kernels (ace_stage.hip, ace_spectral.hip) used by
// ace_pipeline.cpp.  Shapes follow main/src/my_recovery_algorithms/ADMM_v2/
// inferLowRankV4_multi.m: m_t train rows, m_te = m - m_t test rows, r columns.
#pragma once
#include "ace_common.hpp"

namespace ace {

// A_norm = ||A||_F / sqrt(m) with the tol_abs guard (:27-30), one shared A.
void launch_anorm(int m, int n, const double* A, double tol_abs, double* anorm, hipStream_t st);
// dst[i][:] = src[rows[i]][:] / anorm[0]  (complex rows of length n)
void launch_gather_rows(int nrows, int n, const double* src, const int* rows, const double* anorm, double* dst,
                        hipStream_t st);
// B_norm per realisation (:32-35) and Bn = B / B_norm
void launch_bnorm(int m, int batch, const double* B, double tol_abs, double* bnorm, double* Bn, hipStream_t st);
// dst[b][i] = src[b][rows[i]]  (f64)
void launch_gather_b(int m, int nrows, int batch, const double* src, const int* rows, double* dst, hipStream_t st);
// per-realisation blocks of `len` doubles: dst[k] = src[idx[k]] (gather) / dst[idx[k]] = src[k] (scatter)
void launch_move_rows(int count, long long len, const double* src, double* dst, const int* idx, bool scatter,
                      hipStream_t st);
// X[b] (n x r) <- X[b] V, V = eigenvectors of X^H X in ascending order (:263-264)
void launch_gram_rotate(int n, int r, int batch, double* X, int* status, hipStream_t st);
// quality = 1 - ||abs(A_te x) - B_te|| / ||B_te||  (:68)
void launch_quality(int n, int mte, int batch, const double* Ate, const double* X, const double* Bte, double* q,
                    hipStream_t st);
// best of restarts (:79-83): X [b][n], Y [b][m] (c128)
void launch_keep_best(int n, int m, int batch, bool first, const double* q, double* qmax, const double* X,
                      const double* Y, double* Xmax, double* Ymax, hipStream_t st);
// rollback (:89-98) and rescale (:106-107)
void launch_finish(int n, int m, int mt, int batch, const double* qlast, const double* Xr, const double* Yr,
                   const double* Xmax, const double* Ymax, const double* anorm, const double* bnorm, double* Xo,
                   double* Yo, uint32_t* status, hipStream_t st);

// dst[(idx ? idx[k] : k) * ld + col] = src[k] (or_mask 0) or |= src[k] & or_mask, k < count
void launch_put_col(int count, const int* src, const int* idx, int* dst, int ld, int col, unsigned or_mask,
                    hipStream_t st);
// launch_move_rows for rows of `len` bytes (partition tables)
void launch_move_bytes(int count, long long len, const void* src, void* dst, const int* idx, bool scatter,
                       hipStream_t st);
// dst[k] |= bit where flag[k] != 0, k < count
void launch_flag_bits(int count, const unsigned char* flag, int* dst, unsigned bit, hipStream_t st);
void launch_fill(long long count, double v, double* dst, hipStream_t st);

// ---- SpectralInitialize (:561-574) through the m_t x m_t dual Gram (ace_spectral.hip)
// C_b = D_b K D_b with K = A_t A_t^H and D_b = diag(B_t[b][i] / ||a_i||) has the nonzero
// spectrum of As^H As (As = D_b A_t); for an eigenpair (lam, u) of C_b, As^H u is the
// eigenvector of As^H As for lam scaled by sqrt(lam) -- exactly one column of
// X = V(:, 1:r) * diag(sqrt(s(1:r))).  The kernels leave W[b][k] = D_b u_k (k-th largest
// eigenvalue first) and X = A_t^H W is one GEMM over batch*r vectors.
//
// When m_t > n the n x n primal Gram As^H As is the smaller eigenproblem (the driver's large
// sweep points, e.g. m_t = 972 at n = 256): launch_spectral_primal forms it per realisation with
// one batched GEMM (A_t^H weighted by B_i^2/||a_i||^2), symmetrises it as the oracle does, and
// writes X = V(:, 1:r) diag(sqrt(max(0, s))) directly ([batch][r][n]).
bool spectral_primal(int mt, int n);
size_t spectral_scratch_bytes(int mt, int n, int batch, int r);
// pr (per-realisation partitions): K, AH and Bt are the full m-row ones, the rows per realisation in pr
int launch_spectral_primal(int mt, int n, int r, int batch, const double* K, const double* AH, const double* Bt,
                           double* scratch, double* X, int* status, hipStream_t st, const PartRows* pr = nullptr);
int launch_spectral(int mt, int r, int batch, const double* K, const double* Bt, double* scratch, double* W,
                    int* status, hipStream_t st, const PartRows* pr = nullptr);

// ---- batched Hermitian eigenpairs (ace_spectral.hip) for PhaseLift's prox_trace
// (TFOCS/prox_trace.m:88-147) and MyPhaseLift's final eig (MyPhaseLift.m:106-107).
// Each realisation's d x d Hermitian matrix sits in the scratch at `C` (doubles, complex
// row-major) within a per-realisation `stride`; tau != null selects all eigenvalues > tau[b]
// (at most kmax), tau == null the kmax largest; descending.  V [batch][kmax][d] receives
// eigenvector q as row q; the scratch's `misc` slot holds {k_b, sum(lam - tau)}, `lam` the
// eigenvalues.  The matrix is destroyed; realisations with active[b] == 0 are skipped.
struct HeevLayout {
    long long stride, C, misc, lam, dd, ee, z;
};
HeevLayout heev_layout(int d, int kmax);
size_t heev_scratch_bytes(int d, int kmax, int batch);
// path: 0 the unblocked one-stage reduction (hetrd_kernel), 1 the panel-blocked one (hetrd_blk_kernel), 2 the
// two-stage reduction (ace_heev2.hip: dense -> band on the f64 matrix cores, band -> tridiagonal by bulge
// chasing) where heev2_eligible, else 1
// side_ok (tau given, kmax = d): the vectors of the smaller side of tau (misc[2] = 1: those at or below it, see
// trieig_kernel); misc[1] is sum_{lam > tau} (lam - tau) either way
int launch_heev(int d, int kmax, int batch, const double* tau, double* scratch, double* V, int* status,
                const int* active, hipStream_t st, int path = 0, int side_ok = 0);
// the tridiagonal eigenpairs of the reduction's (dd, ee) into z / lam / misc (trieig_kernel, ace_spectral.hip)
void launch_trieig(int d, int kmax, int batch, const double* tau, double* scratch, int* status, const int* active,
                   hipStream_t st, int side_ok);

// ---- two-stage prox eigensolver (ace_heev2.hip): all eigenpairs above tau (kmax = d), 32 <= d <= 256
bool heev2_eligible(int d, int kmax);
size_t heev2_extra_bytes(int d, int batch);   // beyond the one-stage layout's batch * stride
int launch_heev2(int d, int kmax, int batch, const double* tau, double* scratch, double* V, int* status,
                 const int* active, hipStream_t st, int side_ok);

}  // namespace ace
