// Shared definitions for the MI355X (gfx950) 2ACE ADMM kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ace.h"

namespace ace {

using d2 = double2;                                            // one complex128 (re, im)
typedef double d4v __attribute__((ext_vector_type(4)));        // f64 MFMA accumulator

__device__ __forceinline__ d2 cmul(d2 a, d2 b) { return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
__device__ __forceinline__ d2 cmulc(d2 a, d2 b) { /* conj(a) * b */ return make_double2(a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x); }
__device__ __forceinline__ d2 cadd(d2 a, d2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ d2 csub(d2 a, d2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ d2 cscale(d2 a, double s) { return make_double2(a.x * s, a.y * s); }
__device__ __forceinline__ double cabs2(d2 a) { return a.x * a.x + a.y * a.y; }

// Per-realisation solver control block (lives in the workspace).
struct RealState {
    double mu, last_res, opt_obj, nB;
    // written by the Y-step kernel each iteration
    double obj2, nAX2, nY2, nJM2, dY2;
    double pad0, pad1, pad2;
    int32_t iters, done, status, pad3;
};
static_assert(sizeof(RealState) % 16 == 0, "RealState alignment");

// wave64 reduction of a double
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// block reduction of up to NV doubles; all threads get the result. `sh` >= 16*NV doubles.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) sh[w * NV + i] = v[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        double s = 0.0;
        for (int k = 0; k < nw; ++k) s += sh[k * NV + i];
        v[i] = s;
    }
    __syncthreads();
}

// ------------------------------------------------------------------ launchers
// GEMM (MFMA f64) with a shared complex LHS over a batch of realisation vectors:
//   C[b][i] = epi( sum_k op(L)[i][k] * V[b][k] )   (complex)
// mode 0: C = acc, 1: C = E - acc, 2: C = E + acc.  conj_l: use conj(L).
// Batched over `nz` independent problems with strides (complex elements).
void launch_zgemm(int mode, bool conj_l, int M, int K, int nb, const double* L, int ldl, long long strideL,
                  const double* V, int ldv, long long strideV, double* C, const double* E, int ldc,
                  long long strideC, int nz, hipStream_t st);

// Batched GEMV with a private LHS per realisation: C[b] = epi(L_b V[b]) (rows) or
// C[b] = epi(L_b^H V[b]) (cols).  L_b = L + b*strideL (complex M x K row-major).
void launch_zgemv_rows(int mode, int M, int K, int nb, const double* L, long long strideL, const double* V,
                       int ldv, double* C, const double* E, int ldc, hipStream_t st);
void launch_zgemv_cols(int mode, int M, int K, int nb, const double* L, long long strideL, const double* V,
                       int ldv, double* C, const double* E, int ldc, hipStream_t st);

// (I + K)^{-1} in place for `count` m x m HPD matrices (Gauss-Jordan, no pivoting).
void launch_inv_ipk(int m, int count, double* G, long long strideG, hipStream_t st);

// Arguments of the Z-step kernel (ace_zprox.hip).
struct ZArgs {
    int n, m, tx, rx;
    const double* X;   // [b][n] c128
    double* N;         // [b][n]
    double* Z;         // [b][n]  (in: Z0, out: Z)
    double* Q;         // [b][tx*tx] c128 warm-start eigenvectors (may be null)
    RealState* st;
    double* optX;      // [b][n]
    double* optY;      // [b][m]
    const double* Ynew;
    const double* Yold;
    const double* KYnew;
    const double* KYold;
    int* done_count;
    int np;            // rank-profile length
    int rl[4];
    double fl[4];
    double tol_rel, tol_abs, rho;
    int it, fixed_iters, warm, ld_state;
};

void launch_zstep(int variant, bool init, const ZArgs& a, int batch, hipStream_t st);
void launch_zstep1w(bool init, const ZArgs& a, int batch, hipStream_t st);  // A2only, one wave per realisation
void launch_pre(int n, int m, int batch, const double* Z, const double* N, const double* Y, const double* M, double* V,
                double* S, const RealState* rs, hipStream_t st);
void launch_ystep(int m, int batch, const double* S, const double* g, double* M, const double* B, const double* Yold,
                  double* Ynew, RealState* rs, hipStream_t st);
void launch_init(int n, int m, int batch, const double* X0, const double* P0, const double* B, double* X, double* Y,
                 double* M, double* N, RealState* rs, double mu0, hipStream_t st);
void launch_finalize(int n, int m, int batch, const double* optX, const double* optY, const double* Xc,
                     const double* Yc, double* Xo, double* Yo, int32_t* iters, uint32_t* status, double* mu,
                     RealState* rs, hipStream_t st);
void launch_conj_transpose(int rows, int cols, const double* A, double* AH, hipStream_t st);
void launch_synth_codebook(uint64_t seed, long long first, int count, int m, int n, double* A, hipStream_t st);
void launch_synth_channels(uint64_t seed, long long first, int count, int m, int tx, int rx, int L, double snr_db,
                           double x0_noise, const double* A, int a_shared, double* vecH, double* B, double* X0,
                           hipStream_t st);

}  // namespace ace
