// The batched InferADMM driver (main/src/my_recovery_algorithms/ADMM_v2/
// inferLowRankV4_multi.m:281-386), shared by the unit solve (ace_admm_solve_batch,
// r = 1) and the pipeline stages (ace_pipeline.cpp: r = 20 row / column modes of
// inferLowRankImpl :258/:270, and the r = 1 refinement :92/:100).
//
//   setup   K = A A^H, G = (I + K)^{-1}          (replaces U = inv(A'A+I), :242/:286-289)
//   init    :296-310
//   iterate :318-383, one kernel sequence per iteration:
//     pre    V = Z - N/mu, S = Y - M/mu
//     T = S - A V          (MFMA GEMM over batch*r vectors, shared A | GEMV, private A)
//     g = G T
//     ystep  AX = S - g, ArgMinY, M update        (:326-337)
//     KY = K Y                                    (for ||A'Y||, ||A'(Y-Y0)||)
//     X = V + A^H g                               (ArgMinX, :325)
//     zstep  ArgMinZ, N update, residuals, stop test, best tracking, mu update
//   finalize opt_X / opt_Y (:384-385)
#include "ace_host.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>
#include <algorithm>
#include <map>
#include <mutex>

namespace ace {

size_t linops_bytes(bool shared, int batch, int m, int n) {
    Carver cv{nullptr};
    LinOps L;
    linops_carve(cv, shared, batch, m, n, &L);
    return cv.off;
}

void linops_carve(Carver& cv, bool shared, int batch, int m, int n, LinOps* L) {
    const size_t cz = 16, mats = shared ? 1 : (size_t)batch;
    L->shared = shared;
    L->m = m;
    L->n = n;
    L->AH = shared ? cv.take(cz * n * m) : nullptr;
    const bool pc = !shared && pc_supported(m, n);   // room for the private phase-code path
    L->K = cv.take(mats * std::max(cz * m * m, pc ? pc_gw_bytes(m) : 0));
    L->G = cv.take(mats * std::max(cz * m * m, pc ? pc_gt_bytes(m) : 0));
    L->pcodes = pc ? cv.take<uint32_t>(pc_codes_bytes(m, n) * (size_t)batch) : nullptr;
    L->pcb = pc ? cv.take(sizeof(double) * (size_t)batch) : nullptr;
    L->pcflag = pc ? cv.take<int>(sizeof(int)) : nullptr;
    L->pc_ok = false;
    L->batch = batch;
    L->ns = shared ? cv.take(cz * 4 * m * m + 2 * sizeof(double)) : nullptr;
    L->LA8 = shared ? cv.take<int8_t>(i8_frag_bytes(m, n)) : nullptr;
    L->LAH8 = shared ? cv.take<int8_t>(i8_frag_bytes(n, m)) : nullptr;
    L->LK8 = shared ? cv.take<int8_t>(i8k_frag_bytes(m)) : nullptr;
    L->c8 = shared ? cv.take(2 * sizeof(double)) : nullptr;
    L->i8flag = shared ? cv.take<int>(sizeof(int)) : nullptr;
    L->Gf = shared && m <= GYK_MAXM ? cv.take(gyk_gfrag_bytes(m)) : nullptr;
    L->Kfr = shared && m <= GYK_MAXM ? cv.take(gyk_gfrag_bytes(m)) : nullptr;
    L->frag_ok = false;
    L->i8ok = false;
    L->gyk_ok = false;
    L->allow_i8 = true;
}

// A/B and test switches, read from the environment once per solve (tests change them between
// solves in one process; nothing on the iteration path calls getenv):
//   ACE_ZCOMPACT=<it>   from that iteration on the Z-step launches in its compact form
//                       (zstep1w_compact_kernel: one wave per 8 realisations; measured neutral, off)
//   ACE_FUSE=0          the lean Z-step as its own launch instead of in apply_AH's epilogue
//   ACE_GYF=0           gyk_kernel and the fused apply_AH as two launches instead of gyf_kernel
//   ACE_GYF_CTL=0       the Z-step launch, not gyf_kernel, runs the m-space control
//   ACE_MSPACE=0        Z stays in memory through the steady state (no m-space steps, RealState::msp)
//   ACE_MSP_ROOM=<k>    a realisation enters the m-space form only if the perturbation bound would
//                       still hold after k more steps of the current size (default 32)
//   ACE_COLD_SYNC=<k>   the first k iterations of a split solve run all sub-batches' g launches, then
//                       all their Z-steps (cross-stream barriers)
//   ACE_MSP_FAIL_IT=<i> (tests) the perturbation bound of every m-space iterate fails at iteration i,
//                       so the Z-step materialises Z, Z' and opt_X from the implicit form
//   ACE_LAZY_DUAL=0     K Y in gyk_kernel every iteration
//   ACE_LEAN=0          the full one-wave Z-step every iteration (no zlean / certified pass)
//   ACE_NUC_MSP=0       A2nuclear r = 1 in n-space (gyk / apply_AH / Z-step) instead of the m-space
//                       iteration of ace_nucmsp.hip
//   ACE_I8_STAGES=0     the r-column stages' A V, A^H g, K Y as f64 GEMMs instead of int8 digit planes
//   ACE_MSR=0           no m-space runs (msr_kernel): every iteration as its own launches
//   ACE_MSR_START=<it>  first iteration at which an m-space run is tried (default 56)
//   ACE_MSR_RETRY=<k>   after a run stopped early, the next try k iterations after its resume point
//   ACE_MSR_WAVES=4     the m-space run as four waves of four output tiles (default eight of two)
//   ACE_TK_EIG=<it>     the one-wave Z-step takes the full profile's top-K eigenpairs by tridiagonal reduction
//                       (topk_tri) in the init Z-step and iterations <= it; later ones run the warm Jacobi
//                       (default 6; 0: Jacobi throughout); ACE_TK_TRACE=1: its use and fallback counts
//                       on stderr at the end of the solve
//   ACE_I8_COMPACT=1    the fused apply_AH compacts a block's realisations outside the m-space form onto the
//                       first MFMA row tiles (pending its GPU validation: off)
//   ACE_ZCERT=0         the four-wave Z-step (r-column stages) always runs its eigensolver (no Ky Fan
//                       certificate)
struct Knobs {
    int zcompact = 0, cold_sync = 0, msp_fail_it = -1, gyf_ctl = 1, msr_start = 56, msr_retry = 8, msr_waves = 8;
    int tkeig = 6;
    bool tk_trace = false;
    bool msr = true;
    bool fuse = true, gyf = true, mspace = true, lazy_dual = true, lean = true, nuc_msp = true, i8r = true, zcert = true;
    bool r1lz = true;   // rank-one profile: top eigenpair by Lanczos in the one-wave Z-step (ACE_R1_LANCZOS=0: Jacobi)
    double msp_room = 32.0;
};
static Knobs read_knobs() {
    Knobs k;
    const auto on = [](const char* name) {
        const char* e = getenv(name);
        return !(e && e[0] == '0');
    };
    const auto num = [](const char* name, double dflt) {
        const char* e = getenv(name);
        return e ? atof(e) : dflt;
    };
    k.zcompact = (int)num("ACE_ZCOMPACT", 0);
    k.cold_sync = exp_env("ACE_COLD_SYNC") ? atoi(exp_env("ACE_COLD_SYNC")) : 0;
    k.msp_fail_it = (int)num("ACE_MSP_FAIL_IT", -1);
    k.gyf_ctl = (int)num("ACE_GYF_CTL", 1);
    k.msp_room = num("ACE_MSP_ROOM", 32.0);
    k.fuse = on("ACE_FUSE");
    k.gyf = on("ACE_GYF");
    k.mspace = on("ACE_MSPACE");
    k.lazy_dual = on("ACE_LAZY_DUAL");
    k.lean = on("ACE_LEAN");
    k.nuc_msp = on("ACE_NUC_MSP");
    k.i8r = on("ACE_I8_STAGES");
    k.msr = on("ACE_MSR");
    k.zcert = on("ACE_ZCERT");
    k.r1lz = on("ACE_R1_LANCZOS");
    k.tkeig = (int)num("ACE_TK_EIG", 6);
    k.tk_trace = num("ACE_TK_TRACE", 0) != 0;
    k.msr_start = (int)num("ACE_MSR_START", 56);
    k.msr_retry = (int)num("ACE_MSR_RETRY", 8);
    if (k.msr_retry < 1) k.msr_retry = 1;
    k.msr_waves = (int)num("ACE_MSR_WAVES", 8) == 4 ? 4 : 8;
    return k;
}
// ACE_MSR_TRACE=1: one stderr line per m-space run (resume point, steps, exit reasons)
static bool msr_trace() {
    static const bool v = [] {
        const char* e = exp_env("ACE_MSR_TRACE");
        return e && e[0] == '1';
    }();
    return v;
}
// eligibility of the fused kernels: their dynamic LDS within the kernel's derived budget (lds_dyn_budget)
// (the launchers' own rule, lds_ok_budget: a shape within the 64 KiB default needs no attribute)
static bool fuse_ok(const Knobs& k, int m) {
    return k.fuse && lds_ok_budget(i8ah_budget(1), i8ah_lds_bytes(m) + i8ah_fuse_lds_bytes());
}
static bool gyf_ok(const Knobs& k, int m) { return k.gyf && lds_ok_budget(gyf_budget(), gyf_lds_bytes(m)); }

// ACE_NO_I8=1 keeps the f64 matrix-core applies for phase-code codebooks too (A/B comparisons).
static bool i8_disabled() {
    static const bool v = [] {
        const char* e = getenv("ACE_NO_I8");
        return e && e[0] == '1';
    }();
    return v;
}

// Phase-code check and int8 fragment images of A and A^H (ace_i8gemm.hip).
static int i8_setup(LinOps& L, hipStream_t st) {
    const int m = L.m, n = L.n;
    L.i8ok = false;
    if (!L.allow_i8 || i8_disabled()) return ACE_OK;
    ACE_HIP(hipMemsetAsync(L.LA8, 0, i8_frag_bytes(m, n), st));
    ACE_HIP(hipMemsetAsync(L.LAH8, 0, i8_frag_bytes(n, m), st));
    ACE_HIP(hipMemsetAsync(L.i8flag, 0, sizeof(int), st));
    launch_max_abs(2LL * m * n, L.A, L.c8, st);
    launch_i8_expand(m, n, L.A, L.c8, L.LA8, L.LAH8, L.i8flag, st);
    int flag = 1;
    double c[2] = {0.0, 0.0};
    ACE_HIP(read_back(&flag, L.i8flag, sizeof(int), st));
    ACE_HIP(read_back(c, L.c8, sizeof(double), st));
    // apply_AH and K Y both hold the digit planes of an m-long operand in LDS
    L.i8ok = flag == 0 && c[0] > 0.0 && std::isfinite(c[0]) && lds_ok_budget(i8ah_budget(0), i8ah_lds_bytes(m)) &&
             lds_ok_budget(i8ah_budget(2), i8ah_lds_bytes(m));
    if (!L.i8ok) return ACE_OK;
    c[1] = c[0] * c[0];
    ACE_HIP(upload(L.c8 + 1, c + 1, sizeof(double), st));
    ACE_HIP(hipMemsetAsync(L.LK8, 0, i8k_frag_bytes(m), st));
    launch_i8k_expand(m, L.K, L.c8, L.LK8, L.i8flag, st);
    ACE_HIP(read_back(&flag, L.i8flag, sizeof(int), st));
    L.i8ok = flag == 0;
    L.gyk_ok = L.i8ok && L.Gf && lds_ok_budget(gyk_budget(), gyk_lds_bytes(m));
    return ACE_OK;
}

// G = (I + K)^{-1} of the shared K by Newton-Schulz on the matrix cores:
//   X0 = 2/(1 + b) I  with b >= lambda_max(I + K) (Gershgorin) and lambda_min(I + K) >= 1,
//   S_k = I - X_k (I + K),   X_{k+1} = X_k + X_k S_k^H = 2 X_k - X_k (I + K) X_k,
//   then X_{k+1} <- (X_{k+1} + X_{k+1}^H) / 2.
// With X_k exactly Hermitian, S_k^H = I - (I + K) X_k, so this is the self-correcting Schulz step
// (error E -> -E (I + K) E, ||S_{k+1}|| = ||S_k||^2) written in the GEMM's  C = E -/+ V L^H  form.
// (The round-1 form 2X - X X (I + K) is only first-order stable in the part of the rounding error
// that does not commute with I + K: E -> E - (I + K)^-1 E (I + K), which grows like the condition
// number per step -- measured divergence on the reference's 972-row kron-structured train rows.)
// The iteration stops one step after max|S_k| < 1e-10 (the next step's error is ~1e-20, i.e.
// converged to rounding).  A single Gauss-Jordan work-group on one CU took 5.2 ms for m = 256;
// this takes a few dozen small GEMMs.
int ns_inverse(LinOps& L, hipStream_t st) {
    const int m = L.m;
    const long long mm = (long long)m * m;
    double* Ap = L.ns;            // I + K
    double* Id = L.ns + 2 * mm;   // I
    double* R = L.ns + 4 * mm;
    double* Xn = L.ns + 6 * mm;
    double* X = L.G;
    double* flag = L.ns + 8 * mm;   // [0] max|R|, [1] Gershgorin bound (workspace, not a stream-ordered allocation)
    launch_ns_prep(m, L.K, Ap, Id, X, st, flag + 1);
    // The spectrum of I + K lies in [1, b], so ||R_0|| <= rho = (b - 1) / (b + 1) and
    // ||R_k|| <= rho^(2^k): the iteration count that brings max|R_k| below 1e-10 is known from b
    // (one host read instead of a read after every iteration); one more step, as below, and a
    // final check (the polling loop takes over if rounding kept it above the bound).
    double b = 0.0;
    ACE_HIP(read_back(&b, flag + 1, sizeof(double), st));
    int kpred = 60;
    if (std::isfinite(b) && b >= 1.0) {
        const double rho = (b - 1.0) / (b + 1.0);
        kpred = 0;
        for (double e = rho; e >= 1e-10 && kpred < 60; e *= e) ++kpred;
    }
    int it = 0;
    bool done = false;
    auto step = [&]() -> int {
        launch_zgemm(1, true, m, m, m, Ap, m, 0, X, m, 0, R, Id, m, 0, 1, st);   // S = I - X (I+K)
        launch_zgemm(2, true, m, m, m, R, m, 0, X, m, 0, Xn, X, m, 0, 1, st);    // X' = X + X S^H
        launch_hermitize(m, Xn, st);
        std::swap(X, Xn);
        ++it;
        return ACE_OK;
    };
    for (int k = 0; k <= kpred && k < 60; ++k) ACE_TRY(step());   // R_kpred < 1e-10, then one more step
    {   // check R of the last step (it is the residual of the iterate before it: converged one step earlier)
        double h = 0.0;
        launch_max_abs(2 * mm, R, flag, st);
        ACE_HIP(read_back(&h, flag, sizeof(double), st));
        done = h < 1e-10;
    }
    for (; it < 60 && !done;) {   // (rounding kept the residual above the bound: poll as before)
        launch_zgemm(1, true, m, m, m, Ap, m, 0, X, m, 0, R, Id, m, 0, 1, st);
        double h = 0.0;
        launch_max_abs(2 * mm, R, flag, st);
        ACE_HIP(read_back(&h, flag, sizeof(double), st));
        done = h < 1e-10;
        launch_zgemm(2, true, m, m, m, R, m, 0, X, m, 0, Xn, X, m, 0, 1, st);
        launch_hermitize(m, Xn, st);
        std::swap(X, Xn);
        ++it;
    }
#ifdef ACE_DEBUG_SPEC
    fprintf(stderr, "ns_inverse m %d b %g kpred %d it %d done %d\n", m, b, kpred, it, (int)done);
#endif
    if (!done) return fail(ACE_ERR_UNSUPPORTED, "setup: Newton-Schulz inverse of I + K did not converge");
    if (X != L.G) ACE_HIP(hipMemcpyAsync(L.G, X, sizeof(double) * 2 * mm, hipMemcpyDeviceToDevice, st));
    return ACE_OK;
}

// Private phase-code codebooks: code images, then G_b from the exact K_b (ace_private.hip).
// Returns with L.pc_ok = false (and nothing else changed) when some A_b is not a phase code.
static int pc_setup(LinOps& L, int batch, hipStream_t st) {
    const int m = L.m, n = L.n;
    L.pc_ok = false;
    // (the code-image iteration needs the one-wave Z-step that forms X from W = A^H g; the four-wave
    // A/B kernel would make admm_run take the generic path, which reads K and G as matrices)
    if (L.shared || !L.pcodes || !L.allow_i8 || i8_disabled() || !pc_supported(m, n) || batch != L.batch ||
        !zstep_takes_w(ACE_VARIANT_A2ONLY, 1))
        return ACE_OK;
    ACE_HIP(hipMemsetAsync(L.pcflag, 0, sizeof(int), st));
    launch_pc_pack(batch, m, n, L.A, L.pcb, L.pcodes, L.pcflag, st);
    int flag = 1;
    ACE_HIP(read_back(&flag, L.pcflag, sizeof(int), st));
    if (flag != 0) return ACE_OK;
    launch_pc_ginv(batch, m, n, L.pcodes, L.pcb, L.K, L.G, st);
    ACE_LAUNCHED("private setup (code images, G_b)");
    L.pc_ok = true;
    return ACE_OK;
}

int linops_setup(LinOps& L, int batch, hipStream_t st) {
    const int m = L.m, n = L.n;
    const int mats = L.shared ? 1 : batch;
    const long long mm = (long long)m * m, mn = (long long)m * n;
    ProfScope ps(ACE_K_SETUP, st);
    if (!L.shared) {
        ACE_TRY(pc_setup(L, batch, st));
        if (L.pc_ok) return ACE_OK;
    }
    // K[j][i] = sum_k conj(A[i][k]) A[j][k]  : GEMM with L = conj(A), V = rows of A
    launch_zgemm(0, true, m, n, m, L.A, n, mn, L.A, n, mn, L.K, nullptr, m, mm, mats, st);
    if (L.shared) {
        ACE_TRY(ns_inverse(L, st));
    } else {  // one Gauss-Jordan work-group per realisation's matrix (parallel over the batch)
        ACE_HIP(hipMemcpyAsync(L.G, L.K, sizeof(double) * 2 * mm * mats, hipMemcpyDeviceToDevice, st));
        launch_inv_ipk(m, mats, L.G, mm, st);
    }
    if (L.shared) {
        launch_conj_transpose(m, n, L.A, L.AH, st);
        L.frag_ok = L.Gf && L.Kfr;
        if (L.frag_ok) {   // G and K in f64 MFMA fragment order (gyk_kernel, the nuclear m-space iteration)
            launch_gyk_gfrag(m, L.G, L.Gf, st);
            launch_gyk_gfrag(m, L.K, L.Kfr, st);
        }
        ACE_TRY(i8_setup(L, st));
    }
    ACE_LAUNCHED("operator setup (K, G, A^H, fragments, digit planes)");
    return ACE_OK;
}

void admm_state_carve(Carver& cv, int batch, int m, int n, int r, AdmmState* s) {
    const size_t cz = 16, bn = (size_t)batch * r * n, bm = (size_t)batch * r * m;
    s->X = cv.take(cz * bn);
    s->Z = cv.take(cz * bn);
    s->N = cv.take(cz * bn);
    s->V = cv.take(cz * bn);
    s->optX = cv.take(cz * bn);
    s->Q = cv.take(cz * (size_t)batch * 32 * 32);
    s->Z2 = cv.take(cz * (size_t)batch * n);
    s->N2 = cv.take(cz * (size_t)batch * n);
    s->AX = cv.take(cz * (size_t)batch * m);
    for (int i = 0; i < 2; ++i) s->Y[i] = cv.take(cz * bm);
    for (int i = 0; i < 2; ++i) s->KY[i] = cv.take(cz * bm);
    s->M = cv.take(cz * bm);
    s->S = cv.take(cz * bm);
    s->T = cv.take(cz * bm);
    s->g = cv.take(cz * bm);
    s->optY = cv.take(cz * bm);
    s->ypart = cv.take(sizeof(double) * 5 * (size_t)batch * r * ((m + 63) / 64));
    s->st = cv.take<RealState>(sizeof(RealState) * (size_t)batch);
    s->done = cv.take<int>(256);
    s->zeros = cv.take(16 * (size_t)n);
    for (int i = 0; i < 2; ++i) s->Sg[i] = cv.take(cz * bm);
    s->optS = cv.take(cz * bm);
}

// ---- the unit path split into independent sub-batches on concurrent streams.  Each of the four
// kernels of an iteration runs one work-group per CU for ~50-100 us with phases that are either
// memory- or matrix-core-bound; with two sub-batches in flight the Z-step of one (HBM) runs
// beside the GEMMs of the other.  ACE_SPLIT=k selects k sub-batches (default 2, 1 = off).
static int split_count(int batch) {
    static const int v = [] {
        const char* e = getenv("ACE_SPLIT");
        return e ? atoi(e) : 2;
    }();
    int k = v < 1 ? 1 : (v > 4 ? 4 : v);
    while (k > 1 && batch / k < 256) --k;   // keep every sub-batch at least one full wave of CUs
    return k;
}

// AdmmState of realisations [ob, ob + ...) of w (r = 1 layout).  Q is indexed by the Z-step
// kernels with a stride of tx * tx complex per realisation (not the allocation's 32 x 32): the
// warm-start basis must be the one the init Z-step wrote for the same realisation, since the
// perturbation certificate pairs it with that realisation's RealState::kf.
static AdmmState state_slice(const AdmmState& w, long long ob, int m, int n, int tx) {
    AdmmState h = w;
    const long long on = 2 * ob * n, om = 2 * ob * m;
    h.X = w.X + on;
    h.Z = w.Z + on;
    h.N = w.N + on;
    h.Z2 = w.Z2 + on;
    h.N2 = w.N2 + on;
    h.AX = w.AX + om;
    h.V = w.V + on;
    h.optX = w.optX + on;
    h.Q = w.Q + 2 * ob * tx * tx;
    for (int i = 0; i < 2; ++i) {
        h.Y[i] = w.Y[i] + om;
        h.KY[i] = w.KY[i] + om;
    }
    h.M = w.M + om;
    h.S = w.S + om;
    h.T = w.T + om;
    h.g = w.g + om;
    h.optY = w.optY + om;
    h.Sg[0] = w.Sg[0] + om;
    h.Sg[1] = w.Sg[1] + om;
    h.optS = w.optS + om;
    h.st = w.st + ob;
    return h;
}

static int admm_iterate_split(const LinOps& L, const AdmmParams& p, const AdmmState& w, const ZArgs& za0, int batch,
                              const double* B, int nsplit, const Knobs& kn, double* Xo, double* Yo, int32_t* iters,
                              uint32_t* status, double* mu_out, hipStream_t st) {
    const int m = L.m, n = L.n;
    const int chunk = (batch / nsplit + 15) & ~15;
    // The sub-batch streams and fork / join events outlive the solve (one set per device and caller
    // stream): destroying a stream waits for its work, which would make every solve block the host
    // until the GPU finishes it (measured: a 0.7 ms idle gap before the next solve's first kernel).
    // Keyed by (device, caller stream), so solves on different caller streams stay independent; at
    // most kSplitSets sets are kept, the least recently used one is released when a new caller
    // stream needs a set (a caller that makes a stream per solve recycles them).  A set only holds
    // library-owned streams, so a caller stream handle that is destroyed and reused stays correct.
    struct SplitRes {
        hipStream_t s[4] = {};
        hipEvent_t e[4] = {}, c[4] = {};
        unsigned long long used = 0;
    };
    constexpr size_t kSplitSets = 8;
    static std::map<std::pair<int, hipStream_t>, SplitRes> res;
    static unsigned long long tick = 0;
    static std::mutex mtx;
    const auto release = [](SplitRes& r) {
        for (int h = 0; h < 4; ++h) {
            if (r.s[h]) (void)hipStreamDestroy(r.s[h]);
            if (r.e[h]) (void)hipEventDestroy(r.e[h]);
            if (r.c[h]) (void)hipEventDestroy(r.c[h]);
        }
        r = SplitRes{};
    };
    int dev = 0;
    ACE_HIP(hipGetDevice(&dev));
    std::vector<hipStream_t> ss(nsplit, st);
    std::vector<hipEvent_t> ev(nsplit), cev(nsplit);
    {
        std::lock_guard<std::mutex> lk(mtx);
        const auto key = std::make_pair(dev, st);
        auto it = res.find(key);
        if (it == res.end()) {
            if (res.size() >= kSplitSets) {
                auto lru = res.begin();
                for (auto i = res.begin(); i != res.end(); ++i)
                    if (i->second.used < lru->second.used) lru = i;
                release(lru->second);
                res.erase(lru);
            }
            SplitRes r;
            hipError_t e = hipSuccess;
            for (int h = 0; h < 4 && e == hipSuccess; ++h) {
                e = hipEventCreateWithFlags(&r.e[h], hipEventDisableTiming);
                if (e == hipSuccess) e = hipEventCreateWithFlags(&r.c[h], hipEventDisableTiming);
                if (e == hipSuccess) e = hipStreamCreateWithFlags(&r.s[h], hipStreamNonBlocking);
            }
            if (e != hipSuccess) {
                release(r);
                return fail(ACE_ERR_HIP, "sub-batch streams: %s", hipGetErrorString(e));
            }
            it = res.emplace(key, r).first;
        }
        SplitRes& r = it->second;
        r.used = ++tick;
        for (int h = 0; h < nsplit; ++h) {
            ev[h] = r.e[h];
            cev[h] = r.c[h];
            if (h > 0) ss[h] = r.s[h];
        }
    }
    ACE_HIP(hipEventRecord(ev[0], st));   // fork after init
    for (int h = 1; h < nsplit; ++h) ACE_HIP(hipStreamWaitEvent(ss[h], ev[0], 0));
    std::vector<AdmmState> ws(nsplit);
    std::vector<int> nb(nsplit);
    for (int h = 0; h < nsplit; ++h) {
        const long long ob = (long long)h * chunk;
        nb[h] = (int)std::max(0LL, std::min((long long)chunk, batch - ob));
        ws[h] = state_slice(w, ob, m, n, za0.tx);
    }
    // Stagger: sub-batch h >= 1 starts its first iteration once sub-batch 0 has issued `stg`
    // kernels of it, so that the sub-batches run different kernels (HBM- vs matrix-core-bound)
    // side by side instead of the same one (ACE_STAGGER, 0 = start together)
    static const int stg = [] {
        const char* e = exp_env("ACE_STAGGER");
        return e ? atoi(e) : 0;
    }();
    hipEvent_t evs = nullptr;
    if (stg > 0 && nsplit > 1) ACE_HIP(hipEventCreateWithFlags(&evs, hipEventDisableTiming));
    // a refused or failed launch inside the sub-batch loops: the caller's stream still waits for every
    // sub-stream (work already queued there uses the caller's workspace) before the error is returned
    auto split_fail = [&](int lc) -> int {
        for (int h = 1; h < nsplit; ++h)
            if (hipEventRecord(ev[h], ss[h]) == hipSuccess) (void)hipStreamWaitEvent(st, ev[h], 0);
        if (evs) (void)hipEventDestroy(evs);
        return lc;
    };
#define SPLIT_LAUNCHED(stage)                                           \
    do {                                                                \
        const int lc_ = ::ace::launch_check(stage, __FILE__, __LINE__); \
        if (lc_) return split_fail(lc_);                                \
    } while (0)
    auto stagger_mark = [&](int h, int it, int k) -> hipError_t {
        return (evs && h == 0 && it == 1 && k == stg) ? hipEventRecord(evs, ss[0]) : hipSuccess;
    };
    // steady-state Z-steps under the perturbation certificate (zlean_kernel), A2only only
    const bool lean = p.variant != ACE_VARIANT_NUCLEAR && za0.warm && za0.Q && kn.lean;
    // m-space steady state (RealState::msp): needs the fused gyf iteration at every iteration
    const bool msp = lean && za0.lazy_dual && fuse_ok(kn, m) && gyf_ok(kn, m) && kn.mspace;
    const DualCtl dc{za0.tol_abs, za0.tol_rel, za0.rho, za0.fixed_iters, n, 1, w.done};
    // cold iterations (ACE_COLD_SYNC=k: it <= k): the g launches of all sub-batches, then all
    // Z-steps, with a cross-stream barrier after each group, so that no g work-group waits for
    // CUs held by another sub-batch's long cold Z-step
    const int cold_sync = kn.cold_sync;
    auto barrier = [&]() -> int {
        for (int h = 0; h < nsplit; ++h) ACE_HIP(hipEventRecord(cev[h], ss[h]));
        for (int h = 0; h < nsplit; ++h)
            for (int k = 0; k < nsplit; ++k)
                if (k != h) ACE_HIP(hipStreamWaitEvent(ss[h], cev[k], 0));
        return ACE_OK;
    };
    // m-space runs (msr_kernel): from iteration msr_next on, a steady-state block of every sub-batch
    // iterates inside one launch; the per-iteration launches resume where the runs left off
    const bool msr = msp && kn.msr && kn.gyf_ctl && msr_supported(m) && gyf_ok(kn, m) && fuse_ok(kn, m);
    int msr_next = kn.msr_start;
    int q = 0, rc = ACE_OK;
    for (int it = 1; it <= p.maxiter && rc == ACE_OK; ++it) {
        // an m-space run starts only when every live realisation can enter it (a block left out would
        // hold the per-iteration launches for itself while the run occupies the stream): the readiness
        // count is read back (the host waits for iteration it - 1), else the next check comes later
        bool run_msr = false;
        if (msr && it >= msr_next && it < p.maxiter) {
            for (int h = 1; h < nsplit; ++h) {
                ACE_HIP(hipEventRecord(cev[h], ss[h]));
                ACE_HIP(hipStreamWaitEvent(st, cev[h], 0));
            }
            ACE_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(w.done + 28), 0, 3, st));
            launch_msr_ready(batch, w.st, it, w.done + 28, st);
            int nr[3] = {0, 0, 0};
            ACE_HIP(read_back(nr, w.done + 28, sizeof(nr), st));
            run_msr = nr[0] == 0;
            if (msr_trace())
                fprintf(stderr, "msr check it %d: not ready %d (not m-space %d, test pending %d)\n", it, nr[0], nr[1],
                        nr[2]);
            if (!run_msr) msr_next = it + kn.msr_retry;
        }
        if (run_msr) {
            int pidx[4] = {-1, -1, -1, -1};
            for (int h = 0; h < nsplit; ++h) {
                if (nb[h] == 0) continue;
                const AdmmState& wh = ws[h];
                ZArgs za = za0;
                za.it = it;
                za.st = wh.st;
                za.msp = 1;
                za.msp_fail_it = kn.msp_fail_it;
                za.rank_one = za0.rank_one ? za0.rank_one + (long long)h * chunk : nullptr;
                const MsrArgs ma{L.Gf, B + (long long)h * chunk * m, {wh.Y[0], wh.Y[1]}, wh.M, wh.AX,
                                 {wh.Sg[0], wh.Sg[1]}, wh.optS, wh.optY, wh.st, w.done + 8 + h, w.done + 1,
                                 w.done + 12 + 4 * h, msr_trace() ? w.done + 40 + h : nullptr, nb[h], m, it, p.maxiter};
                ACE_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(w.done + 8 + h), p.maxiter, 1, ss[h]));
                ACE_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(w.done + 12 + 4 * h), 0, 4, ss[h]));
                ProfScope ps(ACE_K_MSR, ss[h]);
                pidx[h] = ps.idx;
                launch_msr(ma, za, kn.msr_waves, ss[h]);
                SPLIT_LAUNCHED("m-space run (msr_kernel)");
            }
            for (int h = 1; h < nsplit; ++h) {   // (the caller's stream waits for the sub-batches)
                ACE_HIP(hipEventRecord(cev[h], ss[h]));
                ACE_HIP(hipStreamWaitEvent(st, cev[h], 0));
            }
            int rv[20] = {p.maxiter, p.maxiter, p.maxiter, p.maxiter};   // resume [4], then [4] per sub-batch
            ACE_HIP(read_back(rv, w.done + 8, sizeof(int) * 20, st));
            for (int h = 0; h < nsplit; ++h) {   // algorithmic flops of the run: 8 m^2 per realisation-iteration
                if (pidx[h] >= 0) g_prof.work[pidx[h]] = 8.0 * m * m * rv[4 + 4 * h];
                if (msr_trace())
                    fprintf(stderr, "msr h %d it %d: resume %d steps %d notready %d fail %d pend %d\n", h, it, rv[h],
                            rv[4 + 4 * h], rv[5 + 4 * h], rv[6 + 4 * h], rv[7 + 4 * h]);
            }
            if (msr_trace()) {   // m-vectors written (opt_Y / opt_S and the write-back; cumulative over the solve)
                int vw[4] = {0, 0, 0, 0};
                ACE_HIP(read_back(vw, w.done + 40, sizeof(vw), st));
                fprintf(stderr, "msr it %d: vectors written %d %d %d %d (m = %d)\n", it, vw[0], vw[1], vw[2], vw[3], m);
            }
            int e = p.maxiter;
            for (int h = 0; h < nsplit; ++h)
                if (nb[h] > 0) e = std::min(e, std::max(it, rv[h]));
            it = e;                 // the per-iteration launches run from here (blocks ahead skip)
            q = (it - 1) & 1;
            msr_next = e + kn.msr_retry;
        }
        const bool csync = nsplit > 1 && it <= cold_sync;
      for (int phase = 0; phase < (csync ? 2 : 1); ++phase) {
        const int pmask = csync ? (1 << phase) : 3;   // bit 0: the g launch, bit 1: the Z-step
        for (int h = 0; h < nsplit; ++h) {
            if (nb[h] == 0) continue;
            const AdmmState& wh = ws[h];
            const hipStream_t sh = ss[h];
            if (evs && h > 0 && it == 1) ACE_HIP(hipStreamWaitEvent(sh, evs, 0));
            const double* Bh = B + (long long)h * chunk * m;
            double* Zc = (it & 1) ? wh.Z : wh.Z2;   // Z, N of the previous iterate (ping-pong)
            double* Nc = (it & 1) ? wh.N : wh.N2;
            ACE_HIP(stagger_mark(h, it, 1));
            ZArgs za = za0;
            za.it = it;
            za.wmode = 1;
            za.yfused = 1;
            za.ypart = nullptr;
            za.X = wh.X;
            za.Z = Zc;
            za.N = Nc;
            za.Zn = (it & 1) ? wh.Z2 : wh.Z;
            za.Nn = (it & 1) ? wh.N2 : wh.N;
            za.Q = wh.Q;
            za.st = wh.st;
            za.optX = wh.optX;
            za.optY = wh.optY;
            za.Xcur = wh.V;
            za.Ynew = wh.Y[1 - q];   // (dual_fixup)
            za.Yold = wh.Y[q];
            za.fixup_now = it == p.maxiter;
            za.rank_one = za0.rank_one ? za0.rank_one + (long long)h * chunk : nullptr;
            za.lean = lean;
            za.compact = lean && kn.zcompact > 0 && it > kn.zcompact && it != p.maxiter;
            // the steady-state Z-step in apply_AH's epilogue (not at the last iteration, whose
            // pending convergence tests the one-wave kernels finish, unless m-space steps are on:
            // their realisations have no Z in memory, and the fused control runs dual_fixup)
            za.xfuse = lean && (it != p.maxiter || msp) && fuse_ok(kn, m);
            za.msp = msp;
            za.Af = L.A;
            za.Sold = wh.Sg[(it + 1) & 1];
            za.Snew = wh.Sg[it & 1];
            za.optS = wh.optS;
            za.msp_fail_it = kn.msp_fail_it;
            // and apply_AH in the same launch as gyk (g stays on chip)
            const bool gyf = za.xfuse && za0.lazy_dual && gyf_ok(kn, m);
            GykArgs ga{L.Gf, wh.T, Bh, wh.Y[q], wh.M, wh.Y[1 - q], wh.g, wh.KY[q], wh.KY[1 - q], wh.optY,
                       L.LK8, L.c8, wh.st, wh.AX, 2 - q, L.LA8, Zc, Nc, w.zeros, n, za0.lazy_dual, dc, gyf ? 1 : 0,
                       gyf && msp ? 1 : 0, it, za.Sold, wh.Sg[it & 1], wh.optS, za0.np,
                       {za0.fl[0], za0.fl[1], za0.fl[2], za0.fl[3]}, za.rank_one, kn.msp_room};
            if (!(pmask & 1)) {
            } else if (gyf) {
                ProfScope ps(ACE_K_APPLY_G, sh);
                launch_gyf(nb[h], m, n, ga, L.LAH8, wh.X, za, kn.gyf_ctl, sh);
                SPLIT_LAUNCHED("g / Y-step / apply_AH (gyf_kernel)");
            } else {
                {
                    ProfScope ps(ACE_K_APPLY_G, sh);
                    launch_gyk(nb[h], m, ga, sh);
                }
                SPLIT_LAUNCHED("g / Y-step (gyk_kernel)");
                ACE_HIP(stagger_mark(h, it, 2));
                ProfScope ps(ACE_K_APPLY_AH, sh);
                launch_i8_apply_AH(nb[h], m, n, L.LAH8, wh.g, wh.X, L.c8, wh.st, sh, za.xfuse ? &za : nullptr);
                SPLIT_LAUNCHED("apply_AH (i8ah_kernel)");
            }
            ACE_HIP(stagger_mark(h, it, 3));
            if (pmask & 2) {
                ProfScope ps(ACE_K_ZSTEP, sh);
                if (lean && !za.xfuse) launch_zlean(za, nb[h], sh);
                launch_zstep(p.variant, false, za, nb[h], sh);
                SPLIT_LAUNCHED("Z-step");
            }
        }
        if (csync) ACE_TRY(barrier());
      }
        q = 1 - q;
        if (!p.fixed_iters && (it % 8 == 0) && it < p.maxiter) {
            for (int h = 1; h < nsplit; ++h) {   // (the caller's stream waits for the sub-batches)
                ACE_HIP(hipEventRecord(cev[h], ss[h]));
                ACE_HIP(hipStreamWaitEvent(st, cev[h], 0));
            }
            int h_done = 0;
            ACE_HIP(read_back(&h_done, w.done, sizeof(int), st));
            if (h_done >= batch) break;
        }
    }
    for (int h = 1; h < nsplit; ++h) {   // join
        ACE_HIP(hipEventRecord(ev[h], ss[h]));
        ACE_HIP(hipStreamWaitEvent(st, ev[h], 0));
    }
    ACE_LAUNCHED("split iterations");
#undef SPLIT_LAUNCHED
    {
        ProfScope ps(ACE_K_FINAL, st);
        // best iterates still in m-space form (RealState::optsrc 3): opt_X = Z0 + A^H opt_S
        if (msp) launch_i8_msp_optx(batch, m, n, L.LAH8, w.optS, w.optX, L.c8, w.st, w.Z, w.Z2, w.Sg[0], w.Sg[1], st);
        if (msp && g_prof.on && g_prof.msp_used < g_prof.msp_cap)   // (ace_prof_msp_steps)
            ACE_HIP(hipMemcpyAsync(g_prof.msp_slots + g_prof.msp_used++, w.done + 1, sizeof(int),
                                   hipMemcpyDeviceToHost, st));
        launch_finalize_r(n, m, 1, 1, batch, w.optX, w.optY, w.V, w.Y[q], Xo, Yo, iters, status, mu_out, w.st, st, w.Z,
                          w.Z2, w.Y[0], w.Y[1]);
    }
    ACE_LAUNCHED("finalize (split)");
    if (evs) ACE_HIP(hipEventDestroy(evs));
    return rc;
}

// A2nuclear at r = 1 on a shared A, iterated in m-space (ace_nucmsp.hip): Z and N live as
// (coefficient of X_init, m-vector) pairs; one launch per iteration; X = opt_a X_init + A^H opt_w
// after the loop.  Workspace: zeta, nu in Sg[0], Sg[1], K zeta, K nu in KY[0], KY[1], P0 = A X_init
// in T, opt_w in optS, the last iterate's m-part in g; X_init in X.
static int admm_nuclear_msp(const LinOps& L, const AdmmParams& p, const AdmmState& w, const ZArgs& za0, int batch,
                            const double* B, double* Xo, double* Yo, int32_t* iters, uint32_t* status,
                            double* mu_out, hipStream_t st) {
    const int m = L.m, n = L.n;
    NmsArgs a{};
    a.Gf = L.Gf;
    a.Kf = L.Kfr;
    a.B = B;
    a.M = w.M;
    double *Eb[2] = {w.Sg[0], w.Sg[1]}, *AEb[2] = {w.KY[0], w.KY[1]};   // e, A E ping-pong
    a.Eo = Eb[0];
    a.En = Eb[1];
    a.AEo = AEb[0];
    a.AEn = AEb[1];
    a.P0 = w.T;
    a.optW = w.optS;
    a.optY = w.optY;
    a.curW = w.g;
    a.rs = w.st;
    a.dc = DualCtl{za0.tol_abs, za0.tol_rel, za0.rho, za0.fixed_iters, n, 1, w.done};
    ZArgs za = za0;
    za.lazy_dual = 1;
    {
        ProfScope ps(ACE_K_INIT, st);
        launch_zgemm(0, false, m, n, batch, L.A, n, 0, w.X, n, 0, w.T, nullptr, m, 0, 1, st);   // P0 = A X_init
        launch_nms_init(batch, n, m, w.X, a, st);
    }
    int q = 0, it = 1;
    for (; it <= p.maxiter; ++it) {
        a.Yo = w.Y[q];
        a.Yn = w.Y[1 - q];
        a.Eo = Eb[q];
        a.En = Eb[1 - q];
        a.AEo = AEb[q];
        a.AEn = AEb[1 - q];
        za.it = it;
        {
            ProfScope ps(ACE_K_APPLY_G, st);
            launch_nms(batch, m, a, za, false, st);
        }
        ACE_LAUNCHED("A2nuclear m-space iteration (nms_kernel)");
        q = 1 - q;
        if (!p.fixed_iters && (it % 8 == 0) && it < p.maxiter) {
            int h_done = 0;
            ACE_HIP(read_back(&h_done, w.done, sizeof(int), st));
            if (h_done >= batch) break;
        }
    }
    {
        ProfScope ps(ACE_K_FINAL, st);
        // convergence tests the last iteration left pending (lazy dual residual)
        a.Yo = w.Y[q];
        a.Yn = w.Y[1 - q];
        za.it = std::min(it, p.maxiter);
        launch_nms(batch, m, a, za, true, st);
        launch_nms_out(batch, n, m, w.X, a, w.V, w.g, st);
        // X = a X_init + A^H w  (w.V holds a X_init, w.g the selected m-part)
        launch_zgemm(2, false, n, m, batch, L.AH, m, 0, w.g, m, 0, w.optX, w.V, n, 0, 1, st);
        launch_finalize_r(n, m, 1, 1, batch, w.optX, w.optY, w.optX, w.Y[q], Xo, Yo, iters, status, mu_out, w.st, st,
                          nullptr, nullptr, nullptr, nullptr);
    }
    ACE_LAUNCHED("finalize (A2nuclear m-space)");
    return ACE_OK;
}

// ACE_TK_TRACE: the one-wave Z-step's tridiagonal uses and Jacobi fallbacks (ZArgs::tkcnt) of the solve
static int tk_report(const Knobs& kn, const AdmmState& w, int rc, hipStream_t st) {
    if (!kn.tk_trace || rc != ACE_OK) return rc;
    int tkc[2] = {0, 0};
    ACE_HIP(read_back(tkc, w.done + 32, sizeof(tkc), st));
    fprintf(stderr, "[ace] tridiagonal Z-steps %d, Jacobi fallbacks %d\n", tkc[0], tkc[1]);
    return rc;
}

int admm_run(const LinOps& L, const AdmmParams& p, const AdmmState& w, int batch, const double* B,
             const double* X0, double* Xo, double* Yo, int32_t* iters, uint32_t* status, double* mu_out,
             hipStream_t st) {
    const int m = L.m, n = L.n, r = p.r;
    const Knobs kn = read_knobs();
    if (!L.shared && r != 1) return fail(ACE_ERR_UNSUPPORTED, "private sensing matrices support r = 1 only");
    if (p.part && (r == 1 || !L.shared || p.part->m != m))
        return fail(ACE_ERR_UNSUPPORTED, "per-realisation partitions run the r-column stages on a shared A");
    const int row_mode = (r == 1) ? 1 : p.row_mode;   // the two modes coincide at r = 1
    const int nv = batch * r;                         // vectors per apply
    const long long mm = (long long)m * m, mn = (long long)m * n;
    const bool fast = (r == 1);                       // r = 1 kernels (ystep, one-wave zstep)
    const bool fused = fast && L.shared;              // pre_kernel folded into the shared-A GEMMs
    // phase-code A: int8 digit-plane applies; apply_AH writes W = A^H g and the Z-step forms X
    const bool i8 = fused && L.i8ok && zstep_takes_w(p.variant, r);
    const bool gyk = i8 && L.gyk_ok;                  // g, Y-step, K Y and the dual terms in one kernel
    // private phase-code codebooks: T, g = G T, Y-step, W = A^H g and the dual terms in one kernel
    const bool pc = !L.shared && L.pc_ok && r == 1 && zstep_takes_w(p.variant, r);
    const bool wmode = i8 || pc;
    // r-column stages on a shared phase-code A: A V, A^H g and K Y as exact int8 digit planes over
    // the batch * r vectors (vector j of realisation j / r), G T and the rest unchanged
    const bool i8r = !fast && L.shared && L.i8ok && kn.i8r && nv >= 256;
    g_path[(i8 || i8r) ? 0 : pc ? 1 : L.shared ? 2 : 3].fetch_add(1, std::memory_order_relaxed);
    // pc_ok means K and G hold the code-image path's tiles, not the m x m matrices the generic path reads
    if (L.pc_ok && !pc) return fail(ACE_ERR_UNSUPPORTED, "private phase-code setup without its iteration path");

    auto applyA = [&](int mode, const double* Vin, double* C, const double* E) {  // C = E (-) A Vin
        if (L.shared) launch_zgemm(mode, false, m, n, nv, L.A, n, 0, Vin, n, 0, C, E, m, 0, 1, st);
        else launch_zgemv_rows(mode, m, n, batch, L.A, mn, Vin, n, C, E, m, st);
    };
    auto applyMM = [&](const double* Lm, const double* Vin, double* C) {  // C = L Vin, L = G or K
        if (L.shared) launch_zgemm(0, false, m, m, nv, Lm, m, 0, Vin, m, 0, C, nullptr, m, 0, 1, st);
        else launch_zgemv_rows(0, m, m, batch, Lm, mm, Vin, m, C, nullptr, m, st);
    };
    auto applyAH = [&](const double* gin, double* C, const double* E) {  // C = E + A^H gin
        if (L.shared) launch_zgemm(2, false, n, m, nv, L.AH, m, 0, gin, m, 0, C, E, n, 0, 1, st);
        else launch_zgemv_cols(2, m, n, batch, L.A, mn, gin, m, C, E, n, st);
    };

    ZArgs za{};
    za.n = n;
    za.m = m;
    za.tx = p.tx;
    za.rx = p.rx;
    za.r = r;
    za.row_mode = row_mode;
    za.X = w.X;
    za.N = w.N;
    za.Z = w.Z;
    za.Q = w.Q;
    za.st = w.st;
    za.optX = w.optX;
    za.optY = w.optY;
    za.done_count = w.done;
    za.np = rank_profile(p.prof_tx ? p.prof_tx : p.tx, p.rx, m, p.prof_n ? p.prof_n : n,
                         p.rank_one ? 0 : p.use_rank_one, za.rl, za.fl);
    za.rank_one = p.rank_one;
    za.tol_rel = p.tol_rel;
    za.tol_abs = p.tol_abs;
    za.rho = p.rho;
    za.fixed_iters = p.fixed_iters;
    za.warm = p.eig_warm;
    za.zcert = kn.zcert ? 1 : 0;
    za.mthr = p.part ? p.part->mt : 0;   // thresholds on the realisation's m_t train rows (:364-370)
    za.r1lz = kn.r1lz ? 1 : 0;
    za.tkeig = kn.tkeig > 0 ? kn.tkeig : 0;
    za.tkcnt = w.done + 32;
    za.wmode = 0;
    za.Xcur = w.V;     // wmode: X of never-improved realisations (finalize's fallback)
    za.Zn = nullptr;   // in place (init, and every kernel outside wmode)
    za.Nn = nullptr;
    za.zeros = w.zeros;
    za.nuclear = p.variant == ACE_VARIANT_NUCLEAR;
    // the fused g / Y-step kernel skips K Y; the Z-step forms the dual terms when the convergence
    // test needs them (RealState::dpend), from the shared f64 K
    za.lazy_dual = (gyk && kn.lazy_dual) ? 1 : 0;
    za.Kf = L.K;

    // A2nuclear r = 1 on a shared A: the m-space iteration (ace_nucmsp.hip)
    const bool nms = L.shared && L.frag_ok && r == 1 && p.variant == ACE_VARIANT_NUCLEAR && kn.nuc_msp && nms_supported(m);
    // ---- init (:296-310)
    ACE_HIP(hipMemsetAsync(w.done, 0, 256, st));
    ACE_HIP(hipMemsetAsync(w.zeros, 0, 16 * (size_t)n, st));
    {
        ProfScope ps(ACE_K_INIT, st);
        if (pc) launch_pc_apply_a(batch, m, n, L.pcodes + pc_codesA_off(batch, m, n), L.pcb, X0, w.T, st);
        else applyA(0, X0, w.T, nullptr);                        // AX = A*X0
        launch_init_r(row_mode, n, m, r, batch, X0, w.T, B, w.X, w.Y[0], w.M, w.N, w.st, p.mu0, st, p.part);
        if (!nms) {
            za.it = 0;
            launch_zstep(p.variant, true, za, batch, st);           // Z = ArgMinZ(X, N=0, mu=1)
            if (!pc && !za.lazy_dual) applyMM(L.K, w.Y[0], w.KY[0]); // K*Y (for A'*Y terms; lazy: on demand)
        }
    }
    ACE_LAUNCHED("init (A X0, init, Z-step)");
    if (nms) return admm_nuclear_msp(L, p, w, za, batch, B, Xo, Yo, iters, status, mu_out, st);

    int q = 0;
    const int poll = 8;
    const int nsplit = gyk ? split_count(batch) : 1;
    if (nsplit > 1 || (gyk && kn.mspace && p.variant != ACE_VARIANT_NUCLEAR))
        return tk_report(kn, w, admm_iterate_split(L, p, w, za, batch, B, nsplit, kn, Xo, Yo, iters, status, mu_out, st), st);
    // algorithmic flops of the f64 GEMM-shaped applies as launched (all batch * r vectors; the
    // unit path's fused int8 kernels are accounted by the bench): ace_prof_work
    const double fl_mn = 8.0 * m * n * nv, fl_mm = 8.0 * m * m * nv;
    // ... and their algorithmic HBM bytes (c128 = 16 B; every per-vector array read or written once, a
    // shared operator once per launch) and int8 matrix-core ops (8 digit planes x the 2 x 2 real
    // expansion; K carries two base-128 planes): ace_prof_work_ex, so that the r-column stages' int8
    // applies, Y-step and Z-step get a roofline too
    const double vb = 16.0 * nv;                           // bytes of one c128 entry over the launch's vectors
    const double op_mn = 2.0 * 8 * (2.0 * m) * (2.0 * n) * nv, op_mm = 2.0 * 8 * 2 * (2.0 * m) * (2.0 * m) * nv;
    const double shA = L.shared ? 16.0 * m * n : 16.0 * m * n * batch, shM = L.shared ? 16.0 * m * m : 16.0 * m * m * batch;
    // r-column Z-step: E E^H over the r column blocks (tx x tx x rx r complex MACs) plus the 32 x 32 Hermitian
    // eig (0.8 Mflop at tx = 32); A2nuclear: the r x r Gram E^H E and Z = E V diag V^H
    // (3 n r^2 MACs).  Bytes: X, N, Z in; Z, N out; the warm-start eigenvectors in and out; the dual terms'
    // Y, Y_old, K Y, K Y_old in (m r each)
    const double zs_fl = !fast ? (p.variant == ACE_VARIANT_NUCLEAR
                                      ? 8.0 * 3 * n * r * r * batch
                                      : (8.0 * p.tx * p.tx * p.rx * r + 0.8e6 * std::pow(p.tx / 32.0, 3)) * batch)
                               : 0.0;
    const double zs_b = !fast ? (80.0 * n * r + 64.0 * m * r + 32.0 * p.tx * p.tx) * batch : 0.0;
    // wmode: Z, N ping-pong between (Z, N) and (Z2, N2); the Z-step writes the other pair
    double *Zc = w.Z, *Nc = w.N, *Zo = w.Z2, *No = w.N2;
    double lv = 1.0;   // share of the batch still iterating (convergence mode: from the polls), for ace_prof_work
    for (int it = 1; it <= p.maxiter; ++it) {
        if (pc) {
            ProfScope ps(ACE_K_APPLY_G, st);
            const PgkArgs pa{m, n, L.pcodes, L.pcodes + pc_codesA_off(batch, m, n), L.G, L.pcb, B, w.Y[q], w.M,
                             w.Y[1 - q], w.X, w.optY, w.st, w.AX, 2 - q, Zc, Nc, w.zeros};
            launch_pgk(batch, pa, st);
            ACE_LAUNCHED("private g / Y-step / apply_AH (pgk_kernel)");
        } else if (gyk) {
            // T = (Y - M/mu) - A V is formed inside gyk_kernel (apply_A folded in)
        } else if (i8) {     // T = (Y - M/mu) - A (Z - N/mu), exact digit planes on the int8 matrix cores
            ProfScope ps(ACE_K_APPLY_A, st);
            launch_i8_apply_A(batch, n, m, L.LA8, Zc, Nc, w.Y[q], w.M, w.T, L.c8, w.st, w.zeros, gyk ? w.AX : nullptr, st);
            ACE_LAUNCHED("apply_A (i8a_kernel)");
        } else if (fused) {  // pre_kernel folded into apply_A (V = Z - N/mu, S = Y - M/mu) and apply_AH / ystep
            ProfScope ps(ACE_K_APPLY_A, st, lv * (fl_mn));
            launch_zgemm_fused(true, m, n, batch, L.A, n, w.Z, w.N, n, w.T, w.Y[q], w.M, m, w.st, st);
        } else {
            {
                ProfScope ps(ACE_K_PRE, st, 0.0, lv * (vb * (3.0 * m + (i8r ? 0.0 : 3.0 * n))));
                launch_pre(n * r, m * r, batch, w.Z, w.N, w.Y[q], w.M, i8r ? nullptr : w.V, w.S, w.st, st);
            }
            if (i8r) {   // T = (Y - M/mu) - A (Z - N/mu) per vector, digit planes
                ProfScope ps(ACE_K_APPLY_A, st, 0.0, lv * (vb * (2.0 * n + 3.0 * m)), lv * (op_mn));
                launch_i8_apply_A(nv, n, m, L.LA8, w.Z, w.N, w.Y[q], w.M, w.T, L.c8, w.st, w.zeros, nullptr, st, r);
                ACE_LAUNCHED("r-column apply_A (i8a_kernel)");
            } else {
                ProfScope ps(ACE_K_APPLY_A, st, lv * (fl_mn), lv * (vb * (n + 2.0 * m) + shA));
                applyA(1, w.V, w.T, w.S);   // T = S - A V
            }
        }
        if (pc) {
            // g, the Y-step, W = A^H g and the dual terms came from pgk_kernel
        } else if (gyk) {
            ProfScope ps(ACE_K_APPLY_G, st);
            const GykArgs ga{L.Gf, w.T, B, w.Y[q], w.M, w.Y[1 - q], w.g, w.KY[q], w.KY[1 - q], w.optY, L.LK8, L.c8, w.st,
                             w.AX, 2 - q, L.LA8, Zc, Nc, w.zeros, n, za.lazy_dual,
                             DualCtl{za.tol_abs, za.tol_rel, za.rho, za.fixed_iters, n, 1, w.done}};
            launch_gyk(batch, m, ga, st);
            ACE_LAUNCHED("g / Y-step (gyk_kernel)");
        } else if (fused) {  // g = G T with the Y-step in its epilogue
            ProfScope ps(ACE_K_APPLY_G, st, lv * (fl_mm));
            const YsArgs ys{B, w.Y[q], w.M, w.Y[1 - q], w.ypart};
            launch_zgemm_ystep(m, batch, L.G, w.T, w.g, ys, w.st, st);
        } else {
            {   // g = G T; per-realisation partitions: then (I + K_t)^{-1} T_t by the Schur identity (launch_part_gfix)
                ProfScope ps(ACE_K_APPLY_G, st, lv * (fl_mm), lv * (vb * 2.0 * m + shM) * (p.part ? 2.0 : 1.0));
                applyMM(L.G, w.T, w.g);
                if (p.part) launch_part_gfix(batch, r, *p.part, L.G, w.g, w.st, st);
            }
            {
                ProfScope ps(ACE_K_YSTEP, st, 0.0, lv * (vb * 6.0 * m + 8.0 * m * batch));   // S, g, M, Y in; M, Y' out
                if (fast) launch_ystep(m, batch, w.S, w.g, w.M, B, w.Y[q], w.Y[1 - q], w.st, st);
                else launch_ystep_r(row_mode, m, r, batch, w.S, w.g, w.M, B, w.Y[q], w.Y[1 - q], w.st, st, p.part);
            }
        }
        ACE_LAUNCHED("apply_A / g = G T / Y-step");
        if (!gyk && !pc) {   // K Y
            ProfScope ps(ACE_K_APPLY_K, st, lv * ((i8 || i8r) ? 0.0 : fl_mm), lv * ((i8 && !i8r) ? 0.0 : vb * 2.0 * m + (i8r ? 0.0 : shM)), lv * (i8r ? op_mm : 0.0));
            if (i8) launch_i8_apply_K(batch, m, L.LK8, w.Y[1 - q], w.KY[1 - q], L.c8, w.st, st);
            else if (i8r) launch_i8_apply_K(nv, m, L.LK8, w.Y[1 - q], w.KY[1 - q], L.c8, w.st, st, r);
            else applyMM(L.K, w.Y[1 - q], w.KY[1 - q]);
            ACE_LAUNCHED((i8 || i8r) ? "K Y (i8ah_kernel<KY>)" : "K Y (zgemm)");
        }
        if (!pc) {
            // X = V + A^H g
            ProfScope ps(ACE_K_APPLY_AH, st, lv * ((wmode || i8r) ? 0.0 : fl_mn),
                         lv * (wmode ? 0.0 : i8r ? vb * (m + 3.0 * n) : vb * (m + 2.0 * n) + shA), lv * (i8r ? op_mn : 0.0));
            if (wmode) {
                za.xfuse = gyk && wmode && p.variant != ACE_VARIANT_NUCLEAR && za.warm && za.Q && kn.lean &&
                           it != p.maxiter && fuse_ok(kn, m);
                if (za.xfuse) {   // the fused kernel needs this iteration's Z-step arguments
                    za.it = it;
                    za.wmode = 1;
                    za.Z = Zc;
                    za.N = Nc;
                    za.Zn = Zo;
                    za.Nn = No;
                }
                launch_i8_apply_AH(batch, m, n, L.LAH8, w.g, w.X, L.c8, w.st, st, za.xfuse ? &za : nullptr);
            }
            else if (fused) launch_zgemm_fused(false, n, m, batch, L.AH, m, w.g, nullptr, m, w.X, w.Z, w.N, n, w.st, st);
            else if (i8r) {
                ZArgs zv{};
                zv.r = r;
                zv.xzn = 1;
                zv.Z = w.Z;
                zv.N = w.N;
                zv.zeros = w.zeros;   // (rows of realisations whose N is held as exact zero)
                launch_i8_apply_AH(nv, m, n, L.LAH8, w.g, w.X, L.c8, w.st, st, nullptr, &zv);
            } else applyAH(w.g, w.X, w.V);
            ACE_LAUNCHED((wmode || i8r) ? "apply_AH (i8ah_kernel)" : "apply_AH (zgemm)");
        }
        za.it = it;
        za.wmode = wmode;
        if (wmode) {
            za.Z = Zc;
            za.N = Nc;
            za.Zn = Zo;
            za.Nn = No;
        }
        za.ypart = fused && !gyk ? w.ypart : nullptr;
        za.yfused = gyk || pc;
        za.ytiles = (m + 63) / 64;
        za.Ynew = w.Y[1 - q];
        za.Yold = w.Y[q];
        za.KYnew = w.KY[1 - q];
        za.KYold = w.KY[q];
        za.lean = wmode && p.variant != ACE_VARIANT_NUCLEAR && za.warm && za.Q && kn.lean;
        za.fixup_now = it == p.maxiter;
        za.compact = za.lean && kn.zcompact > 0 && it > kn.zcompact;
        {
            ProfScope ps(ACE_K_ZSTEP, st, lv * (zs_fl), lv * (zs_b));
            if (za.lean && !za.xfuse) launch_zlean(za, batch, st);
            launch_zstep(p.variant, false, za, batch, st);
            ACE_LAUNCHED("Z-step");
        }
        q = 1 - q;
        if (wmode) {
            std::swap(Zc, Zo);
            std::swap(Nc, No);
        }
        if (!p.fixed_iters && (it % poll == 0) && it < p.maxiter) {
            int h_done = 0;
            ACE_HIP(read_back(&h_done, w.done, sizeof(int), st));
            if (h_done >= batch) break;
            lv = (double)(batch - h_done) / batch;
        }
    }
    {
        ProfScope ps(ACE_K_FINAL, st);
        launch_finalize_r(n, m, r, row_mode ? r : 1, batch, w.optX, w.optY, wmode ? w.V : w.X, w.Y[q], Xo, Yo, iters, status,
                          mu_out, w.st, st, wmode ? w.Z : nullptr, wmode ? w.Z2 : nullptr, (gyk || pc) ? w.Y[0] : nullptr,
                          (gyk || pc) ? w.Y[1] : nullptr);
    }
    ACE_LAUNCHED("finalize");
    return tk_report(kn, w, ACE_OK, st);
}

}  // namespace ace
