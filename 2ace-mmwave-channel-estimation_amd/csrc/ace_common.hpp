// Shared definitions for the MI355X (gfx950) 2ACE ADMM kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

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
    // written by the Z-step: upper bound on max|Re|,|Im| of V = Z - N/mu for the next iteration's
    // apply (the exponent of the int8 digit planes, ace_i8gemm.hip); NaN when Z or N is not finite
    double vbound;
    // written by the fused g / Y-step / K Y kernel (ace_i8gemm.hip::gyk_kernel):
    // ||A^H (Y - Y0)||^2 = dY^H (K Y - K Y0) and ||A^H Y||^2 = Y^H K Y
    double dAtY, nAtY;
    int32_t iters, done, status, objcol;  // objcol: argmin column of the per-column objective
    // 1 when the stored N is exactly zero (wmode Z-step, common case Z = E: N + mu (X - Z) is
    // then zero in exact arithmetic and only its rounding residue would be stored); readers use
    // the zero vector instead of N
    int32_t nzero;
    // where opt_X lives: 0 the opt_X buffer; 1 / 2 the Z / Z2 ping-pong buffer (wmode: when the
    // best iterate had N = 0 and Z = E, X = Z' exactly and the copy is deferred until that buffer
    // is about to be overwritten)
    int32_t optsrc;
    // 1 when the next iteration's V = Z - N/mu equals this iteration's X exactly (wmode, N = 0
    // on entry and Z' = E = X): A V is then the AX = (Y - M/mu) - g that gyk_kernel stored, and
    // apply_A skips its product (ace_i8gemm.hip::i8a_kernel)
    int32_t avok;
    // where opt_Y lives (gyk_kernel, like optsrc for opt_X): 0 the opt_Y buffer; 1 / 2 the Y[0] /
    // Y[1] ping-pong buffer holding the best Y_new, copied only before that buffer is overwritten
    int32_t optysrc;
    // Perturbation certificate of the lean Z-step (ace_zprox1w.hip::zlean_kernel).  When the
    // one-wave Z-step's Ky Fan certificate passes with Z' = E (N' = 0), it records for every
    // rank-profile entry p kf[p] = sqrt(sum of the r_p largest row norms^2 of Qprev^H E_ref), a
    // norm of a fixed r_p-row projection of E_ref.  kfcum accumulates ||E_i - E_{i-1}|| over the
    // later iterations, so kf[p] - kfcum bounds that projection of the current E from below
    // (triangle inequality), and by Ky Fan the top-r_p eigenvalue sum of E E^H.  kfok: the bound
    // is valid (the chain E_ref -> E_i has not been broken by a rescaling or N != 0).
    double kf[4];
    double kfcum;
    int32_t kfok;
    int32_t zit;   // iteration whose Z-step the lean kernel completed (the full kernel skips it)
    // Lazy dual residual (ZArgs::lazy_dual): the convergence test (:372) needs res_dual and
    // thresh_dual (the only consumers of A'*Y, :330/:366/:369) only when the primal test passes
    // and the combined one fails.  The Z-step then sets dpend and keeps what dual_fixup needs to
    // finish the test: dZ2 = ||Z - Z0||^2, nZ2 = ||Z||^2 and res_comb.
    double pd_dZ2, pd_nZ2, pd_rc;
    int32_t dpend;
    // the fused apply_AH (ace_i8gemm.hip, i8ah_kernel<false, true>) formed X = Z' of iteration fzit
    // and left ||X||^2 and ||X - Z||^2 for zstep1w_kernel's certificate and iteration control
    int32_t fzit;
    double fs0, fs3;
    // m-space steady state (GykArgs::msp, ace_i8gemm.hip::gyk_body): from iteration it0 on, a
    // certified realisation keeps Z implicit as Z = Z0 + A^H S with S = sum of its g since it0 (Z0
    // the Z buffer z0id = 1 (Z) / 2 (Z2) as it stood at it0).  With N = 0 the fused pass's sums follow
    // from m-space quantities: ||X - Z||^2 = ||A^H g||^2 = g^H K g = Re g^H (T - g) ((I + K) g = T),
    // ||X||^2 = ||Z||^2 + 2 Re (A Z)^H g + ||A^H g||^2 (A Z = A V, the T input), so apply_AH and the
    // Z / Z' traffic drop out of the iteration.  mzit: the iteration gyk_kernel settled that way;
    // msp: the implicit form is live (cleared when the Z-step materialises Z for a full step).
    // optsrc = 3: opt_X = Z0 + A^H opt_S; 4 / 5: the same with opt_S still in the S ping-pong
    // buffer Sg[0] / Sg[1] (deferred like opt_Y: copied only before that buffer is overwritten).
    int32_t msp, mzit, z0id, msp_pad;   // msp_pad: the entry iteration it0
    // m-space run (msr_kernel) that left this realisation's block ahead of the per-iteration launches:
    // the first iteration those must run for the block (its resume point)
    int32_t mres, mres_pad_[3];
    // A2nuclear m-space iteration (ace_nucmsp.hip): E_prev = na X_init + A^H e, Z = naz E_prev,
    // N = nbeta E_prev, nep2 = ||E_prev||^2, nx0 = ||X_init||^2; best / current iterate's X_init coefficient
    double na, nbeta, nx0, nopt_a, ncur_a, naz, nep2, npad2_;
};
static_assert(sizeof(RealState) % 16 == 0, "RealState alignment");

// Parameters of the convergence test (inferLowRankV4_multi.m:364-381) that a deferred dual
// residual needs (ZArgs / GykArgs carry one).
struct DualCtl {
    double tol_abs, tol_rel, rho;
    int fixed_iters, n, r;
    int* done_count;
};
// Finish a convergence test left pending by iter_control (RealState::dpend): res_dual and
// thresh_dual (:366, :369) from dAtY = ||A^H (Y - Y0)||^2 and nAtY = ||A^H Y||^2, the test
// (:372: the primal part held and the combined part failed, so it is the dual part), then the
// stop or the mu update (:379-381).  Returns 1 when the realisation stopped.
__device__ __forceinline__ int dual_finish(const DualCtl& c, RealState* st, double dAtY, double nAtY) {
    const double mu = st->mu, rc = st->pd_rc;
    const double res_dual = mu * sqrt(fmax(0.0, dAtY) + st->pd_dZ2);
    const double t_dual = c.tol_abs * sqrt((double)c.n * c.r * 2) + c.tol_rel * sqrt(fmax(0.0, nAtY) + st->pd_nZ2);
    st->dAtY = dAtY;
    st->nAtY = nAtY;
    st->dpend = 0;
    bool stop = false;
    if (res_dual < t_dual) {
        st->status |= ACE_ST_CONVERGED;
        if (!c.fixed_iters) stop = true;
    }
    if (stop) {
        st->done = 1;
        atomicAdd(c.done_count, 1);
        return 1;
    }
    if (rc > st->last_res * 0.9) st->mu = mu * c.rho;
    st->last_res = rc;
    return 0;
}

// wave64 reduction of a double
// 16-lane butterfly reductions with DPP partners instead of ds_bpermute (__shfl_xor): step o pairs
// lane l with quad_perm l^1, quad_perm l^2, row_half_mirror (7 - l within 8) and row_mirror (15 - l).
// After the steps below o every lane of an o-group holds the same value (x + y == y + x, and max
// likewise, bit for bit), so each partner holds lane l^o's value: the results equal the xor
// butterfly's bit for bit, at VALU latency.
template <int O>
__device__ __forceinline__ double bfly16(double x) {
    constexpr int ctrl = O == 1 ? 0xB1 : O == 2 ? 0x4E : O == 4 ? 0x141 : 0x140;
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), ctrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), ctrl, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double bsum16(double v) {
    v += bfly16<1>(v);
    v += bfly16<2>(v);
    v += bfly16<4>(v);
    v += bfly16<8>(v);
    return v;
}
__device__ __forceinline__ double bmax16(double v) {
    v = fmax(v, bfly16<1>(v));
    v = fmax(v, bfly16<2>(v));
    v = fmax(v, bfly16<4>(v));
    v = fmax(v, bfly16<8>(v));
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

// running max |component| of the entries passed to add(), with a sticky NaN term for
// non-finite entries (fmax alone would drop a NaN)
struct VMax {
    double m = 0.0, s = 0.0;
    __device__ __forceinline__ void add(double2 v) {
        const double ax = fabs(v.x), ay = fabs(v.y);
        m = fmax(m, fmax(ax, ay));
        s += 0.0 * (ax + ay);
    }
};

// wave64 sum with DPP inside the 16-lane rows, one swizzle across the rows of each half, one exchange between the
// halves (VALU latency for 4 of the 6 steps); another association than wave_sum, every lane gets the same value
// x + x[lane ^ 16] and x + x[lane ^ 32] by gfx950's row / half-wave swaps (VALU, no LDS round trip): with both
// operands x, the swap returns the even- and the odd-row (lower- and upper-half) values in every lane, whose sum is
// the pair's sum in the same order in both lanes of a pair
__device__ __forceinline__ double xor16_sum(double v) {
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
    return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double xor32_sum(double v) {
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
    return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
    return xor32_sum(xor16_sum(bsum16(v)));
}
// block_sum with wave_sum_dpp
template <int NV>
__device__ __forceinline__ void block_sum_dpp(double (&v)[NV], double* sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = wave_sum_dpp(v[i]);
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

// block_sum_dpp with one barrier: the caller keeps `sh` barrier-separated from its previous readers and its next
// writers (no barrier before the partials are stored or after they are read)
template <int NV>
__device__ __forceinline__ void block_sum_dpp1(double (&v)[NV], double* sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = wave_sum_dpp(v[i]);
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

// Experiment and diagnostic switches (A/B measurements that were not kept, traces, workspace poisoning):
// read only by a build with -DACE_EXPERIMENTS (make EXTRA=-DACE_EXPERIMENTS); the default build keeps
// their defaults.  The switches the GPU tests use to pin bit-identity between paths stay plain getenv.
inline const char* exp_env(const char* name) {
#ifdef ACE_EXPERIMENTS
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// ------------------------------------------------------------------ dynamic LDS budgets (ace_api.cpp)
// A kernel that takes more dynamic LDS than the 64 KiB default gets its limit raised, once, to the
// CU's 160 KiB less its own static LDS as the code object reports it (hipFuncGetAttributes::
// sharedSizeBytes).  The launchers and the eligibility tests of the paths (ace_admm.cpp, the Z-step
// and spectral launchers) read that one number, so a kernel whose static LDS grows loses the path's
// eligibility (and says so) instead of failing its launches.  0 when the attribute could not be set
// (the HIP error is cleared and the kernel keeps the default budget: no launch above 64 KiB).
constexpr size_t LDS_PER_CU = 160 * 1024;
size_t lds_dyn_budget(const void* kernel);
// A launcher whose dynamic LDS exceeds its kernel's budget does not launch and records it here;
// launch_check (ACE_LAUNCHED, after every stage of a solve) turns that, or a pending HIP launch
// error, into the solve's error naming the stage and the kernel.
void launch_refused(const char* kernel, size_t need, size_t budget);
int launch_check(const char* stage, const char* file, int line);
#define ACE_LAUNCHED(stage)                                                 \
    do {                                                                    \
        const int lc_ = ::ace::launch_check(stage, __FILE__, __LINE__);     \
        if (lc_) return lc_;                                                \
    } while (0)
// true (launch) when need fits the kernel's budget, else records the refusal
bool lds_fits(const void* kernel, const char* name, size_t need);
// the same rule (the 64 KiB default, or the derived budget) without recording anything: for path
// eligibility tests and launchers that have a fallback
bool lds_ok(const void* kernel, size_t need);
bool lds_ok_budget(size_t budget, size_t need);
size_t msr_request_bytes();                  // dynamic LDS of msr_kernel
size_t hetrd_request_bytes(int d, int blk);  // ... of hetrd_kernel (blk = 0) / hetrd_blk_kernel (blk = 1)
size_t heev2_request_bytes(int d, int which);   // ... of he2hb_kernel (0), hb2st_kernel (1), bt2_kernel (2)

// ------------------------------------------------------------------ launchers
// GEMM (MFMA f64) with a shared complex LHS over a batch of realisation vectors:
//   C[b][i] = epi( sum_k op(L)[i][k] * V[b][k] )   (complex)
// mode 0: C = acc, 1: C = E - acc, 2: C = E + acc.  conj_l: use conj(L).
// Batched over `nz` independent problems with strides (complex elements).
// klim (optional): per z-slice bound on the summation index, read from klim[z * klim_stride] (a double, e.g. the
// eigensolver's kept count): operand entries at or beyond it must be zero; their K blocks are skipped
void launch_zgemm(int mode, bool conj_l, int M, int K, int nb, const double* L, int ldl, long long strideL,
                  const double* V, int ldv, long long strideV, double* C, const double* E, int ldc,
                  long long strideC, int nz, hipStream_t st, const double* klim = nullptr, long long klim_stride = 0);

// Batched GEMV with a private LHS per realisation: C[b] = epi(L_b V[b]) (rows) or
// C[b] = epi(L_b^H V[b]) (cols).  L_b = L + b*strideL (complex M x K row-major).
void launch_zgemv_rows(int mode, int M, int K, int nb, const double* L, long long strideL, const double* V,
                       int ldv, double* C, const double* E, int ldc, hipStream_t st);
void launch_zgemv_cols(int mode, int M, int K, int nb, const double* L, long long strideL, const double* V,
                       int ldv, double* C, const double* E, int ldc, hipStream_t st);

// (I + K)^{-1} in place for `count` m x m HPD matrices (Gauss-Jordan, no pivoting).
void launch_inv_ipk(int m, int count, double* G, long long strideG, hipStream_t st);
struct RealState;
void launch_zgemm_fused(bool fv, int M, int K, int nb, const double* L, int ldl, const double* V, const double* V2,
                        int ldv, double* C, const double* E, const double* E2, int ldc, const RealState* rs,
                        hipStream_t st);
// int8 digit-plane applies of a phase-code A (ace_i8gemm.hip)
int i8_nks(int kc);
int i8_ncols(int mc);
size_t i8_frag_bytes(int mc, int kc);
void launch_i8_expand(int m, int n, const double* A, const double* cmax, int8_t* LA, int8_t* LH, int* flag,
                      hipStream_t st);
// T = (Y - M/mu) - c A (Z - N/mu)   (A: m x n phase code, c = *cmax).  With AX != nullptr, a
// 16-realisation block whose realisations all have RealState::avok takes A V = AX (the previous
// Y-step's A X, X = V exactly) and skips the product.
// rcols > 1: nb = batch * rcols vectors, vector j of realisation j / rcols (the r-column stages)
void launch_i8_apply_A(int nb, int n, int m, const int8_t* LA, const double* Z, const double* N, const double* Y,
                       const double* M, double* T, const double* cmax, const RealState* rs, const double* zeros,
                       const double* AX, hipStream_t st, int rcols = 1);
// W = c A^H g  (the Z-step's wmode forms X = (Z - N/mu) + W); needs i8ah_lds_bytes(m) <= i8ah_budget(0)
// fuse != nullptr: the steady-state Z-step runs in the epilogue (i8ah_kernel<false, true>)
struct ZArgs;
void launch_i8_apply_AH(int nb, int m, int n, const int8_t* LAH, const double* g, double* W, const double* cmax,
                        const RealState* rs, hipStream_t st, const ZArgs* fuse = nullptr,
                        const ZArgs* plain = nullptr);
size_t i8ah_lds_bytes(int kc);
size_t i8ah_fuse_lds_bytes();
// dynamic LDS budget (lds_dyn_budget) of i8ah_kernel: kind 0 plain apply_AH, 1 the FUSE form, 2 the K Y form
size_t i8ah_budget(int kind);
// opt_X = Z0 + A^H opt_S for the realisations whose best iterate is in m-space form (optsrc 3;
// Z0 in Zb1 / Zb2 by RealState::z0id), done or not; sets optsrc = 0
void launch_i8_msp_optx(int nb, int m, int n, const int8_t* LAH, const double* optS, double* optX, const double* cmax,
                        RealState* rs, const double* Zb1, const double* Zb2, const double* S0, const double* S1,
                        hipStream_t st);
// Fused g = G T (3M f64 MFMA), Y-step, K Y (int8 digit planes), dual terms and opt_Y for
// 16-realisation blocks (shared phase-code A, r = 1, m <= GYK_MAXM).  Gf: G in f64 MFMA
// fragment order (launch_gyk_gfrag at setup).
constexpr int GYK_MAXM = 256;
size_t gyk_gfrag_bytes(int m);
size_t gyk_lds_bytes(int m);
size_t gyk_budget();   // dynamic LDS budgets (lds_dyn_budget) of gyk_kernel, gyf_kernel
size_t gyf_budget();
void launch_gyk_gfrag(int m, const double* G, double* Gf, hipStream_t st);
struct GykArgs {
    const double* Gf;
    const double* T;
    const double* B;
    const double* Yo;
    double* M;
    double* Yn;
    double* g;
    const double* KYo;
    double* KYn;
    double* optY;
    const int8_t* LK;   // K digit planes (launch_i8k_expand)
    const double* c8;   // c, c^2
    RealState* rs;
    double* AX;         // optional: AX = (Y - M/mu) - g of the Y-step ([nb][m]), apply_A's next A V
    int yn_id;          // 1 + index of Yn in the Y ping-pong pair: opt_Y deferred (RealState::optysrc); 0 = copy
    // apply_A folded in (LA != nullptr): T = (Y - M/mu) - A (Z - N/mu) for blocks with a realisation
    // whose V is not the previous X (RealState::avok), on the int8 matrix cores, straight into LDS
    const int8_t* LA;   // launch_i8_expand image of A
    const double* Z;
    const double* N;
    const double* zeros;
    int n;
    // lazy dual residual: no K Y; a convergence test the previous Z-step left pending
    // (RealState::dpend) is finished at the start from K Y_k and K (Y_k - Y_{k-1}) (Yo, Yn)
    int lazy;
    DualCtl dc;
    int glds;           // (gyf_kernel) g stays in LDS for the fused apply_AH instead of going to a.g
    // m-space steady state (RealState::msp; needs lazy and glds): S' = S + g into Snew (S from Sold,
    // the ping-pong partner), opt_S = S' when the iterate improves, the fused sums into RealState
    int msp;
    int it;
    const double* Sold;
    double* Snew;
    double* optS;
    // the Z-step's rank profile (z_profile): a realisation enters the m-space form only while the
    // perturbation bound has room for `room` more steps of the current size (ACE_MSP_ROOM)
    int np;
    double fl[4];
    const unsigned char* rank_one;
    double room;
};
void launch_gyk(int nb, int m, const GykArgs& a, hipStream_t st);
// gyk + the fused apply_AH (Z-step pass) in one launch; needs a.lazy and a.glds
size_t gyf_lds_bytes(int m);
// ctl = 0: the Z-step launch, not gyf_kernel, runs the m-space control (ACE_GYF_CTL, A/B)
void launch_gyf(int nb, int m, int n, const GykArgs& a, const int8_t* LAH, double* W, const ZArgs& za, int ctl,
                hipStream_t st);
// m-space run (ace_i8gemm.hip::msr_kernel): gyf_kernel's m-space iteration for iterations it0 ..
// it_end - 1 in one launch, per 16-realisation block whose live realisations are all in the m-space
// form; the state is read from / written back to the buffers of the per-iteration launches
// (Y[it & 1], S[it & 1] hold iterate it), and *resume gets the first iteration they must run.
struct MsrArgs {
    const double* Gf;
    const double* B;
    double* Y[2];
    double* M;
    double* AX;
    double* S[2];
    double* optS;
    double* optY;
    RealState* rs;
    int* resume;     // atomicMin target (the caller sets it to it_end)
    int* mspcount;   // m-space step counter (ace_prof_msp_steps)
    int* steps;      // [4]: realisation-iterations this launch ran (bench accounting); blocks not ready,
                     // runs stopped by a failed bound, by a pending test (diagnostics); the caller zeroes them
    int* vecw;       // (nullable) += m-vectors the run wrote to memory: best iterates (opt_Y, opt_S) and the
                     // state written back at a stop (Y twice, M, AX, S twice): its algorithmic write traffic
    int nb, m, it0, it_end;
};
bool msr_supported(int m);
// notready[0] += live realisations of the batch an m-space run from `it` could not take; [1], [2] of
// them not in the m-space form, with a convergence test pending (diagnostics)
void launch_msr_ready(int nb, const RealState* rs, int it, int* notready, hipStream_t st);
void launch_msr(const MsrArgs& a, const ZArgs& za, int waves, hipStream_t st);   // waves: 8 (default) or 4
// KY = K Y with K = c^2 K_int (cmax[1] = c^2): two digit planes of K_int (setup: launch_i8k_expand)
size_t i8k_frag_bytes(int m);
void launch_i8k_expand(int m, const double* K, const double* cmax, int8_t* LK, int* flag, hipStream_t st);
void launch_i8_apply_K(int nb, int m, const int8_t* LK, const double* Y, double* KY, const double* cmax,
                       const RealState* rs, hipStream_t st, int rcols = 1);
// Newton-Schulz start: Ap = I + K, Id = I, X0 = 2/(1 + b) I with b the Gershgorin bound of I + K.
void launch_ns_prep(int m, const double* K, double* Ap, double* Id, double* X0, hipStream_t st, double* bnd);
// out[0] = max |x_i| over n doubles
void launch_max_abs(long long n, const double* x, double* out, hipStream_t st);
// X <- (X + X^H) / 2 for an m x m complex matrix (exactly Hermitian, real diagonal)
void launch_hermitize(int m, double* X, hipStream_t st);

// Private phase-code codebooks (ace_private.hip): 2-bit code images of each A_b, G_b = (I + A_b A_b^H)^{-1}
// as lower 16 x 16 tiles, and the per-realisation iteration kernel (T, g = G T, Y-step, W = A^H g and the
// dual terms on the int8 matrix cores).
constexpr int PC_MAXM = 256, PC_MAXN = 2048;
bool pc_supported(int m, int n);
size_t pc_codes_bytes(int m, int n);             // per realisation (uint32 images)
size_t pc_codesA_off(int batch, int m, int n);   // dword offset of the A images in the batch's code buffer
size_t pc_gw_bytes(int m);                       // Gauss-Jordan workspace per realisation
size_t pc_gt_bytes(int m);                       // G tiles per realisation
// cb[b] = max |component| of A_b; codes; *flag |= 1 unless every entry of every A_b is cb[b] j^k
void launch_pc_pack(int batch, int m, int n, const double* A, double* cb, uint32_t* codes, int* flag, hipStream_t st);
// Gw <- I + A A^H (exact from the codes), inverted in place; Gt <- its lower tiles
void launch_pc_ginv(int batch, int m, int n, const uint32_t* codes, const double* cb, double* Gw, double* Gt,
                    hipStream_t st);
struct PgkArgs {
    int m, n;
    const uint32_t* codesH;   // A^H images of the batch (launch_pc_pack)
    const uint32_t* codesA;   // A images (codes + pc_codesA_off)
    const double* Gt;
    const double* cb;
    const double* B;
    const double* Yo;
    double* M;
    double* Yn;
    double* W;                // [b][n] c128 out: W = A^H g (the Z-step's wmode forms X)
    double* optY;
    RealState* rs;
    double* AX;
    int yn_id;                // as GykArgs::yn_id
    const double* Z;          // V = Z - N/mu for the cold A V
    const double* N;
    const double* zeros;
};
void launch_pgk(int batch, const PgkArgs& a, hipStream_t st);
// P0 = A X0 (init, InferADMM :296-300) from the code images (codesA = codes + pc_codesA_off)
void launch_pc_apply_a(int batch, int m, int n, const uint32_t* codesA, const double* cb, const double* X0, double* P0,
                       hipStream_t st);

// A2nuclear r = 1 in m-space on a shared A (ace_nucmsp.hip): per-realisation m-vectors, c128
// [batch][m]; Gf, Kf: G = (I + K)^-1 and K = A A^H in f64 MFMA fragment order (launch_gyk_gfrag).
struct NmsArgs {
    const double* Gf;
    const double* Kf;
    const double* B;
    const double* Yo;   // Y of the previous iterate (read)
    double* Yn;         // Y_new (written)
    double* M;
    double* Eo;         // e of E_prev = na X_init + A^H e (read)
    double* En;         // e of E_new (written; Eo / En ping-pong)
    double* AEo;        // A E_prev (read)
    double* AEn;        // A E_new (written)
    const double* P0;   // A X_init (init only)
    double* optW;       // best iterate X = nopt_a X_init + A^H optW
    double* optY;
    double* curW;       // the last iterate's m-part while no objective was finite
    RealState* rs;
    DualCtl dc;
};
size_t nms_lds_bytes(int m);
bool nms_supported(int m);   // nms_lds_bytes(m) within the kernels' LDS budgets
// fin: only finish the convergence tests the previous (last) iteration left pending
void launch_nms(int nb, int m, const NmsArgs& a, const ZArgs& za, bool fin, hipStream_t st);
void launch_nms_init(int nb, int n, int m, const double* Xi, const NmsArgs& a, hipStream_t st);
void launch_nms_out(int nb, int n, int m, const double* Xi, const NmsArgs& a, double* V, double* Wsel, hipStream_t st);

// Arguments of the Z-step kernel (ace_zprox.hip).
struct ZArgs {
    int n, m, tx, rx;
    int r;             // columns per realisation: X, N, Z are [b][r][n], Y, KY [b][r][m]
    int row_mode;      // scale_by_row: objective over all rows (1) or per column with argmin (0)
    const double* X;   // [b][r][n] c128
    double* N;         // [b][r][n]
    double* Z;         // [b][r][n]  (in: Z0, out: Z)
    double* Q;         // [b][tx*tx] c128 warm-start eigenvectors (may be null)
    RealState* st;
    double* optX;      // [b][row_mode ? r : 1][n]
    double* optY;      // [b][row_mode ? r : 1][m]
    const double* Ynew;
    const double* Yold;
    const double* KYnew;
    const double* KYold;
    int* done_count;
    int np;            // rank-profile length (use_rank_one = 0)
    int rl[4];
    double fl[4];
    const unsigned char* rank_one;  // per-realisation use_rank_one (null: all 0); profile [1], [0.95]
    double tol_rel, tol_abs, rho;
    int it, fixed_iters, warm, ld_state;
    // Y-step reductions left as per-tile partials by the fused apply_G epilogue (null: the
    // ystep kernel wrote them to RealState): ypart[(b * ytiles + t) * 5 + k], k = obj2, nAX2,
    // nY2, nJM2, dY2
    const double* ypart;
    int ytiles;
    // wmode (A2only r = 1, non-init): the X buffer holds W = A^H g, and the Z-step forms
    // X = (Z - N/mu) + W itself (xw below); X of realisations that never improved goes to Xcur
    int wmode;
    double* Xcur;
    // outputs Z', N' (null: in place).  When distinct from Z, N (ping-pong, r = 1) the one-wave
    // kernel writes the common-case outputs Z' = E, N' = N + mu (X - E) as it forms E, and only
    // rewrites them when the tail rescaling fires.
    double* Zn;
    double* Nn;
    // the Y-step sums, the dual terms (RealState::dAtY, nAtY) and opt_Y come from gyk_kernel
    int yfused;
    const double* zeros;   // n zero complex entries (the N of realisations with nzero set)
    int nuclear;           // one-wave kernel: A2nuclear r = 1 prox Z = E max(0, |E| - 1/mu) / |E|
    int lean;              // zlean_kernel ran before this launch: skip realisations with st->zit == it
    // lazy dual residual (RealState::dpend): the dual terms are formed only when the convergence
    // test needs them, from the f64 K = A A^H (shared, [m][m] c128) and Ynew, Yold
    int lazy_dual;
    const double* Kf;
    int fixup_now;   // last iteration: finish a pending test here (dual_fixup), no later gyk_kernel
    int xfuse;       // the fused apply_AH ran: realisations with st->fzit == it have X in Zn and their sums
    int compact;     // steady state: zstep1w_compact_kernel (one wave per 8 realisations)
    // m-space steady state (RealState::msp): realisations with st->mzit == it were settled by
    // gyk_kernel (no apply_AH pass); a failed bound materialises Z, Z' (and opt_X) from Af, S
    int msp;
    const double* Af;      // A [m][n] c128
    const double* Sold;
    const double* Snew;
    const double* optS;
    int matz;              // (launch_i8_msp_optx) the apply_AH launch forms opt_X = Z0 + A^H opt_S
    int msp_fail_it;       // (tests: ACE_MSP_FAIL_IT) the bound of m-space iterates fails at this iteration
    int xzn;               // (apply_AH of the r-column stages) write X = (Z - N/mu) + A^H g instead of W
    int zcert;             // four-wave A2only Z-step: skip the eigensolver when the Ky Fan certificate holds
    int r1lz;              // one-wave Z-step: rank-one profile realisations take the top eigenpair by Lanczos
                           // (r1_top, ace_zprox1w.hip) instead of the full Jacobi eigensolver
    int mthr;              // rows of the convergence thresholds (:364-370) when they differ from the state's m:
                           // per-realisation train partitions keep m-space state, the reference's A_t has m_t rows
    int tkeig;             // one-wave Z-step, full profile: the top-K eigenpairs by tridiagonal reduction (topk_tri,
                           // ace_zprox1w.hip) in the init Z-step and iterations it <= tkeig (0: Jacobi throughout)
    int* tkcnt;            // (diagnostics, nullable) [2]: topk_tri uses, and fallbacks to the Jacobi eigensolver
};
// X = V + W with V = Z - N/mu, the one rounding sequence used by every producer of X in wmode
__device__ __forceinline__ double2 xw(double2 z, double2 n, double2 w, double imu) {
    return make_double2(fma(-n.x, imu, z.x) + w.x, fma(-n.y, imu, z.y) + w.y);
}
// Y-step fused into the g = G T epilogue (r = 1, shared G): ArgMinY, M update, Y_new and the
// five reductions as per-(realisation, 64-output tile) partials.
struct YsArgs {
    const double* B;   // [b][m]
    const double* Yo;  // [b][m] c128 (Y of the previous iterate: S = Yo - M/mu)
    double* M;         // [b][m] c128 in/out
    double* Yn;        // [b][m] c128 out
    double* part;      // [b][tilesI][5]
};
void launch_zgemm_ystep(int m, int nb, const double* G, const double* T, double* g, const YsArgs& ys,
                        const RealState* rs, hipStream_t st);

void launch_zstep(int variant, bool init, const ZArgs& a, int batch, hipStream_t st);
// Z_b = U soft(S, tau) V^H of the n x r matrices E_b ([b][r][n] c128, r <= 32): the r-general
// nuclear Z-prox kernel in its init form.  Returns 0 or a hipError_t.
int launch_nuclear_prox(int batch, int n, int r, const double* E, double tau, double* Z, hipStream_t st);
bool zstep_takes_w(int variant, int r);

// ArgMinZ rank profile of realisation b (inferLowRankV4_multi.m:437-464; use_rank_one -> :448-450).
struct ZProfile {
    int np;
    int rl[4];
    double fl[4];
};
__device__ __forceinline__ ZProfile z_profile_flag(const ZArgs& a, int rank_one_b) {   // rank_one[b] given
    ZProfile p;
    if (rank_one_b) {
        p.np = 1;
        p.rl[0] = 1;
        p.fl[0] = 0.95;
        for (int i = 1; i < 4; ++i) { p.rl[i] = 0; p.fl[i] = 0.0; }
    } else {
        p.np = a.np;
        for (int i = 0; i < 4; ++i) { p.rl[i] = a.rl[i]; p.fl[i] = a.fl[i]; }
    }
    return p;
}
__device__ __forceinline__ ZProfile z_profile(const ZArgs& a, int b) {
    return z_profile_flag(a, a.rank_one ? (int)a.rank_one[b] : 0);
}
void launch_zstep1w(bool init, const ZArgs& a, int batch, hipStream_t st);  // A2only, one wave per realisation
// steady-state A2only Z-step (wmode, ping-pong, N = 0 on entry) under the perturbation
// certificate (RealState::kf); realisations it cannot certify are left to launch_zstep1w
void launch_zlean(const ZArgs& a, int batch, hipStream_t st);
void launch_pre(int n, int m, int batch, const double* Z, const double* N, const double* Y, const double* M, double* V,
                double* S, const RealState* rs, hipStream_t st);
void launch_ystep(int m, int batch, const double* S, const double* g, double* M, const double* B, const double* Yold,
                  double* Ynew, RealState* rs, hipStream_t st);
// r-column stage kernels (ace_stage.hip).  State is [b][r][n] / [b][r][m].
// init: InferADMM :296-310 given P0 = A X0 (row mode: one scale, normalize_rows by row
// norms; column mode: per-column scale and entrywise normalisation).
// Per-realisation train / test partitions of the r-column stages (MATLAB's randsample inside every
// inferLowRankV4_multi call, :48-53).  The stage state stays in m-space: every shared-A product runs on
// the full (normalised) A, the test rows of Y and M are held at zero, and g = (I + K_t)^{-1} T_t comes
// from the full G = (I + K)^{-1} by the Schur identity (I + K_tt)^{-1} = G_tt - G_te G_ee^{-1} G_et
// (launch_part_gfix); only the m_te x m_te block G_ee^{-1} is per realisation.
struct PartRows {
    const int* rows;             // [nb][m]: train rows in sampled order, then the test rows ascending
    const unsigned char* mask;   // [nb][ldmask]: 1 on train rows
    const double* geinv;         // [nb][mte][mte] c128: G_ee^{-1}
    int m, mt, ldmask;
};
constexpr int PART_MAXTE = 96;   // test rows per realisation the LDS inverse takes (m <= 1920 at cc_frac 0.95)
void launch_init_r(int row_mode, int n, int m, int r, int batch, const double* X0, const double* P0,
                   const double* B, double* X, double* Y, double* M, double* N, RealState* rs, double mu0,
                   hipStream_t st, const PartRows* pr = nullptr);
// ystep at r columns (ArgMinY :511-533 row / column mode, M update, reductions, and
// in column mode the per-column objective with its first argmin, :352-361).
void launch_ystep_r(int row_mode, int m, int r, int batch, const double* S, const double* g, double* M,
                    const double* B, const double* Yold, double* Ynew, RealState* rs, hipStream_t st,
                    const PartRows* pr = nullptr);
// G_ee^{-1} per realisation from the full G (m x m, row-major c128); status |= ACE_ST_EIG_NOCONV on a
// non-positive pivot (G_ee is a principal block of an HPD matrix: cannot happen in exact arithmetic)
void launch_part_geinv(int nb, const PartRows& pr, const double* G, double* geinv, int* status, hipStream_t st);
// g[b][j] (m-space, = G T~ on entry) <- (I + K_t)^{-1} T_t on the train rows, 0 on the test rows
void launch_part_gfix(int nb, int r, const PartRows& pr, const double* G, double* g, const RealState* rs,
                      hipStream_t st);
// dst[b][j][rows[k]] = src[b][j][k] (k < mt), 0 on the test rows: compact (sampled order) -> m-space
void launch_part_expand(int nb, int r, const PartRows& pr, const double* src, double* dst, hipStream_t st);
// dst[b][j][k] = src[b][j][rows[k]], k < mt: m-space -> compact
void launch_part_compact(int nb, int r, const PartRows& pr, const double* src, double* dst, hipStream_t st);
// quality (:68) with A the full normalised A and B the full normalised B, on each realisation's test rows
void launch_part_quality(int n, int nb, const PartRows& pr, const double* A, const double* X, const double* B,
                         double* q, hipStream_t st);
// opt_X / opt_Y (nc columns) or, if the objective never was finite, the current iterate.
void launch_finalize_r(int n, int m, int r, int nc, int batch, const double* optX, const double* optY,
                       const double* Xc, const double* Yc, double* Xo, double* Yo, int32_t* iters,
                       uint32_t* status, double* mu, RealState* rs, hipStream_t st,
                       const double* Zb1 = nullptr, const double* Zb2 = nullptr, const double* Yb1 = nullptr,
                       const double* Yb2 = nullptr);
void launch_conj_transpose(int rows, int cols, const double* A, double* AH, hipStream_t st);
void launch_synth_codebook(uint64_t seed, long long first, int count, int m, int n, double* A, hipStream_t st);
void launch_synth_channels(uint64_t seed, long long first, int count, int m, int tx, int rx, int L, double snr_db,
                           double x0_noise, const double* A, int a_shared, double* vecH, double* B, double* X0,
                           hipStream_t st);

}  // namespace ace
