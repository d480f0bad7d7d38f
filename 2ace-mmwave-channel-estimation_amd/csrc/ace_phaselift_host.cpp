// C-ABI of the batched PhaseLift solver: ace_phaselift_solve_batch replaces
// recoveredSig = MyPhaseLift(measurements, measurementMat)
// (main/src/my_recovery_algorithms/MyPhaseLift.m:69-107) for a batch of measurement vectors
// sharing one measurement matrix.  The TFOCS iteration (kernels in ace_phaselift.hip) runs in
// the reduced coordinates of range(Phi^H); this file sets the reduction up (Phi Phi^H = R^H R),
// drives tfocs_AT.m's outer / inner loops over the batch and maps the leading eigenvector back.
#include <cstring>

#include "ace_host.hpp"
#include "ace_phaselift.hpp"

using namespace ace;

namespace {

struct PlDims {
    int batch, m, n, d, reduced;
};

struct PlWs {
    double *K, *R, *RT, *AH, *T, *wfin, *tau;
    int* ok;
    PlArgs a;
};

void pl_carve(Carver& cv, const PlDims& D, PlWs* w) {
    const size_t cz = 16, B = (size_t)D.batch, dd = (size_t)D.d * D.d;
    w->K = cv.take(cz * (size_t)D.m * D.m);
    w->R = D.reduced ? cv.take(cz * (size_t)D.d * D.m) : nullptr;
    w->RT = cv.take(cz * (size_t)D.m * D.d);
    w->AH = cv.take(cz * (size_t)D.n * D.m);
    w->T = cv.take(cz * B * D.d * D.m);
    w->wfin = cv.take(cz * B * D.d);
    w->ok = cv.take<int>(256);
    PlArgs& a = w->a;
    double** mats[] = {&a.x, &a.xo, &a.z, &a.zo, &a.y, &a.G, &a.Znew, &a.P, &a.VT, &a.V};
    for (double** p : mats) *p = cv.take(cz * B * dd);
    double** vecs[] = {&a.Ax, &a.Axo, &a.Az, &a.Azo, &a.Ay, &a.gAy, &a.gAx, &a.Aex};
    for (double** p : vecs) *p = cv.take(8 * B * D.m);
    a.Pg = cv.take(cz * B * D.d * D.m);
    a.st = cv.take<PlState>(sizeof(PlState) * B);
    a.act = cv.take<int>(4 * B);
    a.cnt = cv.take<int>(256);
    a.tau = cv.take(8 * B);
    a.hl = heev_layout(D.d, D.d);
    a.scratch = cv.take(heev_scratch_bytes(D.d, D.d, D.batch));
}

int validate(const ace_phaselift_cfg* c, int batch, int m, int n, PlDims* D) {
    if (!c) return fail(ACE_ERR_ARG, "cfg is NULL");
    if (batch < 1 || m < 1 || n < 1) return fail(ACE_ERR_ARG, "batch/m/n must be >= 1 (got %d/%d/%d)", batch, m, n);
    if (c->maxIts < 1 || c->restart == 0 || c->cntr_reset < 0) return fail(ACE_ERR_ARG, "bad maxIts/restart/cntr_reset");
    if (!(c->lambda > 0)) return fail(ACE_ERR_ARG, "lambda must be > 0 (prox_trace.m:36)");
    if (!(c->beta > 0 && c->beta < 1) || !(c->alpha > 0) || !(c->L0 > 0))
        return fail(ACE_ERR_ARG, "need 0 < beta < 1, alpha > 0, L0 > 0");
    const int d = m <= n ? m : n;
    if (d > 1600) return fail(ACE_ERR_UNSUPPORTED, "min(m, n) = %d > 1600 (eigensolver LDS limit)", d);
    *D = PlDims{batch, m, n, d, m <= n};
    return ACE_OK;
}

}  // namespace

extern "C" {

void ace_phaselift_cfg_default(ace_phaselift_cfg* c) {
    std::memset(c, 0, sizeof *c);
    c->maxIts = 4000;        // MyPhaseLift.m:82
    c->restart = 200;        // :84
    c->cntr_reset = 50;      // tfocs_initialize: round(abs(-50)) (10 when tol < 1e-12)
    c->tol = 1e-10;          // :83
    c->lambda = 5e-2;        // :91
    c->L0 = 1.0;             // tfocs_initialize defaults
    c->alpha = 0.9;
    c->beta = 0.5;
}

size_t ace_phaselift_workspace_size(const ace_phaselift_cfg* cfg, int batch, int m, int n) {
    PlDims D;
    const std::string keep = g_err;
    if (validate(cfg, batch, m, n, &D)) {
        g_err = keep;
        return 0;
    }
    Carver cv{nullptr};
    PlWs w;
    pl_carve(cv, D, &w);
    return cv.off + 256;
}

}  // extern "C"

namespace {
// ace_phaselift_solve_batch; Xout (device, may be NULL): the final TFOCS iterate [batch][d][d] (reduced coordinates)
int solve_batch(const ace_phaselift_cfg* cfg, int batch, int m, int n, const double* Phi, const double* bvec,
                double* sig, int32_t* iters, uint32_t* status, void* workspace, size_t workspace_bytes, void* stream,
                double* Xout) {
    PlDims D;
    ACE_TRY(validate(cfg, batch, m, n, &D));
    if (!Phi || !bvec || !sig || !workspace) return fail(ACE_ERR_ARG, "NULL buffer");
    hipStream_t st = (hipStream_t)stream;
    {
        Carver sz{nullptr};
        PlWs w0;
        pl_carve(sz, D, &w0);
        if (sz.off + 256 > workspace_bytes)
            return fail(ACE_ERR_WORKSPACE, "workspace too small: need %zu bytes, got %zu", sz.off + 256, workspace_bytes);
    }
    poison_workspace(workspace, workspace_bytes, st);
    Carver cv{(char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255)};
    PlWs w;
    pl_carve(cv, D, &w);
    const int d = D.d;
    PlArgs& a = w.a;
    a.d = d;
    a.m = m;
    a.batch = batch;
    a.cntr_reset = cfg->tol < 1e-12 ? 10 : cfg->cntr_reset;
    a.restart = cfg->restart < 0 ? -cfg->restart : cfg->restart;
    a.maxIts = cfg->maxIts;
    a.lambda = cfg->lambda;
    a.alpha = cfg->alpha;
    a.beta = cfg->beta;
    a.Lexact = INFINITY;
    a.tol = cfg->tol;
    a.L0 = cfg->L0;
    a.bvec = bvec;

    // ---- reduction: Phi^H = Q R (m <= n: R = chol(Phi Phi^H)), else Q = I, R = Phi^H
    {
        ProfScope ps(ACE_K_SETUP, st);
        launch_conj_transpose(m, n, Phi, w.AH, st);
        if (D.reduced) {
            launch_zgemm(0, true, m, n, m, Phi, n, 0, Phi, n, 0, w.K, nullptr, m, 0, 1, st);   // K = Phi Phi^H
            launch_chol(m, w.K, w.R, w.ok, st);
            int ok = 0;
            ACE_HIP(read_back(&ok, w.ok, sizeof(int), st));
            if (!ok) return fail(ACE_ERR_UNSUPPORTED, "measurement matrix rows are linearly dependent (Phi Phi^H "
                                 "not positive definite); the reduced PhaseLift needs rank(Phi) = m <= n");
            a.R = w.R;
        } else {
            a.R = w.AH;
        }
        launch_ztranspose(d, m, a.R, w.RT, st);
    }
    // ---- tfocs_initialize: x0 = y = z = 0, A vectors 0
    const size_t dd = 16 * (size_t)batch * d * d, vm = 8 * (size_t)batch * m;
    for (double* p : {a.x, a.xo, a.z, a.zo, a.y, a.G}) ACE_HIP(hipMemsetAsync(p, 0, dd, st));
    for (double* p : {a.Ax, a.Axo, a.Az, a.Azo, a.Ay, a.Aex}) ACE_HIP(hipMemsetAsync(p, 0, vm, st));
    ACE_HIP(hipMemsetAsync(a.cnt, 0, 256, st));
    if (status) ACE_HIP(hipMemsetAsync(status, 0, 4 * (size_t)batch, st));
    launch_pl_init(a, st);
    ACE_LAUNCHED("PhaseLift init");

    auto applyA = [&](const double* X, double* out) {  // out = A(X) = diag(R^H X R), active rows only
        launch_zgemm(0, false, m, d, batch * d, w.RT, d, 0, X, d, 0, w.T, nullptr, m, 0, 1, st);
        launch_pl_diagform(d, m, batch, a.R, w.T, out, a.act, st);
    };
    // the prox's reduction (launch_heev's path): the two-stage one (ace_heev2.hip, r06) where it applies, else the
    // panel-blocked one-stage hetrd_blk_kernel; ACE_HETRD_BLK=0 / 1 / 2 selects the unblocked / blocked one-stage /
    // two-stage reduction (A/B and the GPU tests that pin the paths against each other), read once per solve
    const char* hb = getenv("ACE_HETRD_BLK");
    const int path = hb && hb[0] == '0' ? 0 : (hb && hb[0] == '1' ? 1 : 2);
    // ACE_PROX_SIDE=1: the prox's eigenvectors from the smaller side of the threshold (trieig_kernel).  Off by
    // default: at config 4 the pairs at or below the threshold form large near-zero clusters, and their
    // orthogonalisation in trieig costs more than the back-transform saves (r06: 69.7 vs 81.1 rec/s)
    const char* sd = getenv("ACE_PROX_SIDE");
    const int side_ok = sd && sd[0] == '1';
    const int blk = path == 0 ? 0 : 1;   // (the final top-1 eig: one-stage)
    int h[8];
    for (int outer = 0; outer < cfg->maxIts + 1; ++outer) {
        launch_pl_outer_begin(a, st);
        for (;;) {  // tfocs_AT.m inner (backtracking) loop, for the realisations still in it
            ACE_HIP(hipMemsetAsync(a.cnt, 0, 8 * sizeof(int), st));
            launch_pl_theta(a, st);
            ACE_HIP(read_back(h, a.cnt, sizeof h, st));
            if (h[0] == 0) break;
            {
                ProfScope ps(ACE_K_PRE, st);
                launch_pl_make_y(a, st);
                if (h[1]) applyA(a.y, a.Aex);
                launch_pl_set_Ay(a, st);
                launch_pl_grad(a, st);
            }
            // algorithmic flops per realisation still in the inner loop (h[0]): A*(g) = R diag(g) R^H
            // (8 d^2 m), the prox's dense Hermitian eigendecomposition (17.3 d^3, SURVEY.md §8d's
            // count for eig with vectors), its assembly V diag(s) V^H (8 d^3), A(z) (8 m d^2)
            const double act = h[0], dd3 = (double)d * d * d, dd2m = (double)d * d * m;
            if (h[4]) {  // g_y = A*(g_Ay) = R diag(g) R^H
                ProfScope ps(ACE_K_APPLY_AH, st, 8.0 * dd2m * act);
                launch_zgemm(0, true, d, m, batch * d, a.R, m, 0, a.Pg, m, 0, a.G, nullptr, d, 0, 1, st);
            }
            {
                ProfScope ps(ACE_K_ZSTEP, st, 17.3 * dd3 * act);   // prox_trace: eig of z_old - step g_y, shrink
                launch_pl_prox_in(a, st);
                ACE_TRY(launch_heev(d, d, batch, a.tau, a.scratch, a.V, (int*)status, a.act, st, path, side_ok));
                launch_pl_assemble(a, st);
            }
            {
                ProfScope ps(ACE_K_APPLY_G, st, 8.0 * dd3 * act);   // z = V diag(s) V^H
                // (summation over the kept pairs only: P's and VT's columns q >= k are zero, misc[0] = k)
                launch_zgemm(0, true, d, d, d, a.VT, d, (long long)d * d, a.P, d, (long long)d * d, a.Znew, nullptr, d,
                             (long long)d * d, batch, st, a.scratch + a.hl.misc, a.hl.stride);
                launch_pl_take_z(a, st);
            }
            { ProfScope ps(ACE_K_APPLY_A, st, 8.0 * dd2m * act); applyA(a.z, a.Az); }
            {
                ProfScope ps(ACE_K_YSTEP, st);
                launch_pl_make_x(a, st);
                ACE_HIP(read_back(&h[2], a.cnt + 2, sizeof(int), st));
                if (h[2]) {
                    applyA(a.x, a.Aex);
                    launch_pl_set_Ax(a, st);
                }
                launch_pl_backtrack(a, st);
            }
            ACE_LAUNCHED("PhaseLift inner iteration");
        }
        launch_pl_iterate(a, st);   // tfocs_iterate.m: stopping tests, restart
        int ndone = 0;
        ACE_HIP(read_back(&ndone, a.cnt + 8, sizeof(int), st));
        if (ndone >= batch) break;
    }
    // ---- MyPhaseLift.m:106-107: leading eigenvector of X, scaled by sqrt of its eigenvalue
    {
        ProfScope ps(ACE_K_FINAL, st);
        const HeevLayout h1 = heev_layout(d, 1);
        launch_pl_final_in(d, batch, a.x, a.scratch, h1, st);
        ACE_TRY(launch_heev(d, 1, batch, nullptr, a.scratch, a.V, (int*)status, nullptr, st, blk));
        launch_pl_final_vec(d, batch, D.reduced, a.R, a.V, a.scratch, h1, D.reduced ? w.wfin : sig, st);
        if (D.reduced)   // sig = Phi^H w,  w = R^{-1} sig_d
            launch_zgemm(0, false, n, m, batch, w.AH, m, 0, w.wfin, m, 0, sig, nullptr, n, 0, 1, st);
        launch_pl_outputs(batch, a.st, iters, status, st);
    }
    if (Xout) ACE_HIP(hipMemcpyAsync(Xout, a.x, 16 * (size_t)batch * d * d, hipMemcpyDeviceToDevice, st));
    ACE_LAUNCHED("PhaseLift final eigenvector");
    return ACE_OK;
}

int solve_host(const ace_phaselift_cfg* cfg, int batch, int m, int n, const double* Phi, const double* bvec,
               double* sig, int32_t* iters, uint32_t* status, double* Xr) {
    g_err.clear();
    PlDims D;
    ACE_TRY(validate(cfg, batch, m, n, &D));
    const size_t nP = 16 * (size_t)m * n, nb = 8 * (size_t)batch * m, ns = 16 * (size_t)batch * n,
                 nx = 16 * (size_t)batch * D.d * D.d, ws = ace_phaselift_workspace_size(cfg, batch, m, n);
    std::vector<void*> bufs;
    auto cleanup = [&]() {
        for (void* q : bufs) (void)hipFree(q);
        bufs.clear();
    };
    auto dalloc = [&](size_t bytes, void** q) -> hipError_t {
        hipError_t e = hipMalloc(q, bytes);
        if (e == hipSuccess) bufs.push_back(*q);
        return e;
    };
    void *dP, *db, *ds, *di, *dst, *dw, *dx = nullptr;
    hipError_t e;
    if ((e = dalloc(nP, &dP)) || (e = dalloc(nb, &db)) || (e = dalloc(ns, &ds)) || (e = dalloc(4 * (size_t)batch, &di)) ||
        (e = dalloc(4 * (size_t)batch, &dst)) || (e = dalloc(ws, &dw)) || (Xr && (e = dalloc(nx, &dx)))) {
        cleanup();
        return fail(ACE_ERR_HIP, "hipMalloc: %s", hipGetErrorString(e));
    }
    if ((e = hipMemcpy(dP, Phi, nP, hipMemcpyHostToDevice)) || (e = hipMemcpy(db, bvec, nb, hipMemcpyHostToDevice))) {
        cleanup();
        return fail(ACE_ERR_HIP, "hipMemcpy: %s", hipGetErrorString(e));
    }
    int rc = solve_batch(cfg, batch, m, n, (const double*)dP, (const double*)db, (double*)ds, (int32_t*)di,
                         (uint32_t*)dst, dw, ws, nullptr, (double*)dx);
    if (rc == ACE_OK) {
        if ((e = hipDeviceSynchronize()) || (e = hipMemcpy(sig, ds, ns, hipMemcpyDeviceToHost)) ||
            (iters && (e = hipMemcpy(iters, di, 4 * (size_t)batch, hipMemcpyDeviceToHost))) ||
            (status && (e = hipMemcpy(status, dst, 4 * (size_t)batch, hipMemcpyDeviceToHost))) ||
            (Xr && (e = hipMemcpy(Xr, dx, nx, hipMemcpyDeviceToHost))))
            rc = fail(ACE_ERR_HIP, "phaselift: %s", hipGetErrorString(e));
    }
    const std::string keep = g_err;
    cleanup();
    g_err = keep;
    return rc;
}
}  // namespace

extern "C" {

int ace_phaselift_solve_batch(const ace_phaselift_cfg* cfg, int batch, int m, int n, const double* Phi,
                              const double* bvec, double* sig, int32_t* iters, uint32_t* status, void* workspace,
                              size_t workspace_bytes, void* stream) {
    g_err.clear();
    return solve_batch(cfg, batch, m, n, Phi, bvec, sig, iters, status, workspace, workspace_bytes, stream, nullptr);
}

int ace_phaselift_solve_host(const ace_phaselift_cfg* cfg, int batch, int m, int n, const double* Phi,
                             const double* bvec, double* sig, int32_t* iters, uint32_t* status) {
    return solve_host(cfg, batch, m, n, Phi, bvec, sig, iters, status, nullptr);
}

int ace_phaselift_solve_host_x(const ace_phaselift_cfg* cfg, int batch, int m, int n, const double* Phi,
                               const double* bvec, double* sig, int32_t* iters, uint32_t* status, double* Xr) {
    if (!Xr) {
        g_err.clear();
        return fail(ACE_ERR_ARG, "NULL buffer");
    }
    return solve_host(cfg, batch, m, n, Phi, bvec, sig, iters, status, Xr);
}

int ace_prox_eig_host(int batch, int d, int path, const double* A, const double* tau, double* lam, double* V,
                      int32_t* k) {
    g_err.clear();
    if (batch < 1 || d < 2 || d > 1600 || !A || !tau || !lam || !V || !k) return fail(ACE_ERR_ARG, "bad ace_prox_eig_host arguments");
    const HeevLayout hl = heev_layout(d, d);
    const size_t dd = 16 * (size_t)d * d, sb = heev_scratch_bytes(d, d, batch);
    void *ds = nullptr, *dt = nullptr, *dv = nullptr;
    auto cleanup = [&]() {
        for (void* q : {ds, dt, dv}) (void)hipFree(q);
    };
    hipError_t e;
    if ((e = hipMalloc(&ds, sb)) || (e = hipMalloc(&dt, 8 * (size_t)batch)) || (e = hipMalloc(&dv, dd * batch))) {
        cleanup();
        return fail(ACE_ERR_HIP, "hipMalloc: %s", hipGetErrorString(e));
    }
    double* sc = (double*)ds;
    int rc = ACE_OK;
    for (int b = 0; b < batch && !rc; ++b)
        if ((e = hipMemcpy(sc + (size_t)b * hl.stride + hl.C, A + 2 * (size_t)b * d * d, dd, hipMemcpyHostToDevice)))
            rc = fail(ACE_ERR_HIP, "hipMemcpy: %s", hipGetErrorString(e));
    if (!rc && (e = hipMemcpy(dt, tau, 8 * (size_t)batch, hipMemcpyHostToDevice)))
        rc = fail(ACE_ERR_HIP, "hipMemcpy: %s", hipGetErrorString(e));
    if (!rc) rc = launch_heev(d, d, batch, (const double*)dt, sc, (double*)dv, nullptr, nullptr, nullptr, path & 3, path >> 2);
    if (!rc) rc = launch_check("prox eig", __FILE__, __LINE__);
    if (!rc && (e = hipDeviceSynchronize())) rc = fail(ACE_ERR_HIP, "prox eig: %s", hipGetErrorString(e));
    if (!rc && (e = hipMemcpy(V, dv, dd * batch, hipMemcpyDeviceToHost))) rc = fail(ACE_ERR_HIP, "hipMemcpy: %s", hipGetErrorString(e));
    for (int b = 0; b < batch && !rc; ++b) {
        double misc[3] = {0.0, 0.0, 0.0};
        if ((e = hipMemcpy(misc, sc + (size_t)b * hl.stride + hl.misc, 24, hipMemcpyDeviceToHost)) ||
            (e = hipMemcpy(lam + (size_t)b * d, sc + (size_t)b * hl.stride + hl.lam, 8 * (size_t)d, hipMemcpyDeviceToHost)))
            rc = fail(ACE_ERR_HIP, "hipMemcpy: %s", hipGetErrorString(e));
        k[b] = misc[2] != 0.0 ? -(int32_t)misc[0] : (int32_t)misc[0];
    }
    const std::string keep = g_err;
    cleanup();
    g_err = keep;
    return rc;
}

}  // extern "C"
