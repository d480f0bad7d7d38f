// Device state and launchers of the batched PhaseLift / TFOCS-AT solver (ace_phaselift.hip,
// driven by ace_phaselift_host.cpp).  All matrices are in the reduced coordinates (d x d,
// complex row-major, one per realisation); vectors of A(.) values are real [batch][m].
#pragma once
#include "ace_common.hpp"
#include "ace_pipe.hpp"

namespace ace {

// TFOCS scalars of one realisation (names follow tfocs_AT.m / tfocs_backtrack.m / tfocs_iterate.m)
struct PlState {
    double L, L_old, theta, theta_old;
    double f_x, f_y, C_x, C_z;
    double cntr_Ax, cntr_Ay;         // doubles: tfocs_backtrack sets cntr_Ax = Inf to force a reset
    double xy_sq, nx2, ndx2, dot_xy_g;
    double localL, step;
    int32_t n_iter, restart_iter, backtrack_simple, backtrack_steps;
    int32_t have_gAy, have_gy, have_gAx, ycomp;
    int32_t need_Ay, need_Ax, inner, done;
    int32_t status, pad[3];
};

struct PlArgs {
    int d, m, batch;
    int cntr_reset, restart, maxIts;
    double lambda, alpha, beta, Lexact, tol, L0;
    double *x, *xo, *z, *zo, *y, *G, *Znew, *P, *VT, *V;   // [batch][d][d] c128
    double *Ax, *Axo, *Az, *Azo, *Ay, *gAy, *gAx, *Aex;    // [batch][m] f64
    const double* bvec;                                    // [batch][m] f64
    const double* R;                                       // [d][m] c128 (Phi^H = Q R)
    double* Pg;                                            // [batch][d][m] c128  R o g
    PlState* st;
    int* act;                                              // [batch] in the current inner step
    int* cnt;   // per inner step: [0] active [1] A_y exact [2] A_x exact [4] new g_y; [8] done (whole run)
    double* scratch;                                       // eigensolver scratch (HeevLayout hl)
    HeevLayout hl;
    double* tau;                                           // [batch] lambda * step
};

void launch_pl_init(const PlArgs& a, hipStream_t st);
void launch_pl_outer_begin(const PlArgs& a, hipStream_t st);
void launch_pl_theta(const PlArgs& a, hipStream_t st);
void launch_pl_make_y(const PlArgs& a, hipStream_t st);
void launch_pl_set_Ay(const PlArgs& a, hipStream_t st);
void launch_pl_grad(const PlArgs& a, hipStream_t st);
void launch_pl_prox_in(const PlArgs& a, hipStream_t st);
void launch_pl_assemble(const PlArgs& a, hipStream_t st);
void launch_pl_take_z(const PlArgs& a, hipStream_t st);
void launch_pl_make_x(const PlArgs& a, hipStream_t st);
void launch_pl_set_Ax(const PlArgs& a, hipStream_t st);
void launch_pl_backtrack(const PlArgs& a, hipStream_t st);
void launch_pl_iterate(const PlArgs& a, hipStream_t st);
// a[b][i] = Re sum_r conj(R[r][i]) T[b][r][i]  (A(X) = diag(R^H X R) from T = X R)
void launch_pl_diagform(int d, int m, int batch, const double* R, const double* T, double* out, const int* act,
                        hipStream_t st);
void launch_pl_outputs(int batch, const PlState* st, int32_t* iters, uint32_t* status, hipStream_t s);
void launch_chol(int m, const double* K, double* R, int* ok, hipStream_t st);
void launch_ztranspose(int rows, int cols, const double* S, double* D, hipStream_t st);
void launch_pl_final_in(int d, int batch, const double* x, double* scratch, HeevLayout hl, hipStream_t st);
void launch_pl_final_vec(int d, int batch, int reduced, const double* R, const double* V1, const double* scratch,
                         HeevLayout hl, double* out, hipStream_t st);

}  // namespace ace
