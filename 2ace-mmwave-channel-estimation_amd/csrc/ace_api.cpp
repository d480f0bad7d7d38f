// C-ABI (include/ace.h) of the MI355X 2ACE ADMM hot path: the unit solve
// ace_admm_solve_batch (InferADMM at r = 1, main/src/my_recovery_algorithms/ADMM_v2/
// inferLowRankV4_multi.m:281-386, driven by admm_run in ace_admm.cpp), its host-buffer
// wrapper, synthetic traces, kernel timing, error text and version.
#include <algorithm>
#include <cstring>
#include <mutex>
#include <unordered_map>

#include "ace_host.hpp"

using namespace ace;

namespace {
int cols(const ace_admm_cfg* c) { return c->r == 0 ? 1 : c->r; }   // r = 0: the refinement stage, r = 1

int validate(const ace_admm_cfg* c, int batch, int m, int n, int tx, int rx) {
    if (!c) return fail(ACE_ERR_ARG, "cfg is NULL");
    if (batch < 1 || m < 1 || n < 1) return fail(ACE_ERR_ARG, "batch/m/n must be >= 1 (got %d/%d/%d)", batch, m, n);
    if (tx * rx != n) return fail(ACE_ERR_ARG, "n (%d) != tx*rx (%d*%d)", n, tx, rx);
    if (c->variant != ACE_VARIANT_A2ONLY && c->variant != ACE_VARIANT_NUCLEAR)
        return fail(ACE_ERR_ARG, "unknown variant %d", c->variant);
    if (c->variant == ACE_VARIANT_A2ONLY && (tx < 1 || tx > 32 || ((tx & 1) && tx > 31) || rx > 32))
        return fail(ACE_ERR_UNSUPPORTED, "A2only Z-prox needs tx in [1,32] and rx <= 32 (got %d, %d)", tx, rx);
    if (n > 4096 || m > 4096) return fail(ACE_ERR_UNSUPPORTED, "m, n must be <= 4096 (got %d, %d)", m, n);
    if (c->maxiter < 1) return fail(ACE_ERR_ARG, "maxiter must be >= 1");
    if (!(c->mu0 > 0) || !(c->rho > 0)) return fail(ACE_ERR_ARG, "mu0 and rho must be > 0");
    const int r = cols(c);
    if (r < 1 || r > 32) return fail(ACE_ERR_UNSUPPORTED, "r must be in [1, 32] (got %d)", r);
    if (r > 1 && !c->a_shared) return fail(ACE_ERR_UNSUPPORTED, "r > 1 needs a shared A (a_shared = 1)");
    return ACE_OK;
}
}  // namespace

namespace ace {
namespace {
std::mutex g_lds_mu;
std::unordered_map<const void*, size_t> g_lds_budget;
thread_local std::string t_refused;   // the first launch a launcher refused since the last launch_check
}  // namespace

size_t lds_dyn_budget(const void* kernel) {
    std::lock_guard<std::mutex> lk(g_lds_mu);
    const auto it = g_lds_budget.find(kernel);
    if (it != g_lds_budget.end()) return it->second;
    hipFuncAttributes fa{};
    size_t budget = 0;
    if (hipFuncGetAttributes(&fa, kernel) == hipSuccess && fa.sharedSizeBytes < LDS_PER_CU) {
        const size_t want = LDS_PER_CU - fa.sharedSizeBytes;
        if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)want) == hipSuccess)
            budget = want;
    }
    (void)hipGetLastError();   // (a failed query or setter leaves no sticky error behind)
    g_lds_budget.emplace(kernel, budget);
    return budget;
}

void launch_refused(const char* kernel, size_t need, size_t budget) {
    if (!t_refused.empty()) return;
    char buf[256];
    snprintf(buf, sizeof buf, "%s not launched: %zu B of dynamic LDS requested, budget %zu B", kernel, need, budget);
    t_refused = buf;
}

bool lds_ok_budget(size_t budget, size_t need) { return need <= 64 * 1024 || need <= budget; }
bool lds_ok(const void* kernel, size_t need) {
    return need <= 64 * 1024 || need <= lds_dyn_budget(kernel);   // (the default limit needs no attribute)
}
bool lds_fits(const void* kernel, const char* name, size_t need) {
    if (lds_ok(kernel, need)) return true;
    launch_refused(name, need, lds_dyn_budget(kernel));
    return false;
}

int launch_check(const char* stage, const char* file, int line) {
    if (!t_refused.empty()) {
        const std::string why = t_refused;
        t_refused.clear();
        (void)hipGetLastError();
        return fail(ACE_ERR_UNSUPPORTED, "%s: %s (%s:%d)", stage, why.c_str(), file, line);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(ACE_ERR_HIP, "%s: launch failed: %s (%s:%d)", stage, hipGetErrorString(e), file, line);
    return ACE_OK;
}
}  // namespace ace

extern "C" {

const char* ace_last_error(void) { return g_err.c_str(); }
const char* ace_version(void) { return "ace-mi355x 0.1.0 (gfx950)"; }

int ace_lds_request(const char* kernel, int m, size_t* bytes) {
    g_err.clear();
    if (!kernel || !bytes || m < 1) return fail(ACE_ERR_ARG, "bad ace_lds_request arguments");
    const std::string k = kernel;
    if (k == "i8ah" || k == "i8ah_ky") *bytes = i8ah_lds_bytes(m);
    else if (k == "i8ah_fuse") *bytes = i8ah_lds_bytes(m) + i8ah_fuse_lds_bytes();
    else if (k == "gyk") *bytes = gyk_lds_bytes(m);
    else if (k == "gyf") *bytes = gyf_lds_bytes(m);
    else if (k == "msr") *bytes = msr_request_bytes();
    else if (k == "nms") *bytes = nms_lds_bytes(m);
    else if (k == "hetrd") *bytes = hetrd_request_bytes(m, 0);
    else if (k == "hetrd_blk") *bytes = hetrd_request_bytes(m, 1);
    else if (k == "he2hb") *bytes = heev2_request_bytes(m, 0);
    else if (k == "hb2st") *bytes = heev2_request_bytes(m, 1);
    else if (k == "bt2") *bytes = heev2_request_bytes(m, 2);
    else return fail(ACE_ERR_ARG, "unknown kernel '%s'", kernel);
    return ACE_OK;
}

int ace_prof_sample(int stride, uint32_t full_mask) {
    g_err.clear();
    if (stride < 1) return fail(ACE_ERR_ARG, "stride must be >= 1");
    g_prof.stride = stride;
    g_prof.full = full_mask;
    return ACE_OK;
}

int ace_prof_start(int max_launches) {
    g_err.clear();
    if (max_launches < 1) return fail(ACE_ERR_ARG, "max_launches must be >= 1");
    for (hipEvent_t e : g_prof.ev) (void)hipEventDestroy(e);
    g_prof.ev.assign(2 * (size_t)max_launches, nullptr);
    for (auto& e : g_prof.ev) ACE_HIP(hipEventCreate(&e));
    g_prof.cls.assign(max_launches, 0);
    g_prof.work.assign(max_launches, 0.0);
    g_prof.wbytes.assign(max_launches, 0.0);
    g_prof.wops.assign(max_launches, 0.0);
    g_prof.used = 0;
    for (int& c : g_prof.seen) c = 0;
    if (!g_prof.msp_slots) {
        g_prof.msp_cap = 4096;
        ACE_HIP(hipHostMalloc(reinterpret_cast<void**>(&g_prof.msp_slots), sizeof(int) * g_prof.msp_cap));
    }
    g_prof.msp_used = 0;
    g_prof.on = true;
    return ACE_OK;
}

int ace_prof_msp_steps(long long* steps) {
    g_err.clear();
    if (!steps) return fail(ACE_ERR_ARG, "steps is NULL");
    *steps = g_prof.msp_total;
    return ACE_OK;
}

int ace_prof_work(double* flops) {
    g_err.clear();
    if (!flops) return fail(ACE_ERR_ARG, "flops is NULL");
    for (int c = 0; c < ACE_NKCLASS; ++c) flops[c] = g_prof.work_tot[c];
    return ACE_OK;
}

int ace_prof_work_ex(double* flops, double* bytes, double* int8_ops) {
    g_err.clear();
    for (int c = 0; c < ACE_NKCLASS; ++c) {
        if (flops) flops[c] = g_prof.work_tot[c];
        if (bytes) bytes[c] = g_prof.bytes_tot[c];
        if (int8_ops) int8_ops[c] = g_prof.ops_tot[c];
    }
    return ACE_OK;
}

int ace_path_counts(int64_t* counts, int reset) {
    g_err.clear();
    for (int k = 0; k < 4; ++k) {
        const long long v = reset ? g_path[k].exchange(0) : g_path[k].load();
        if (counts) counts[k] = v;
    }
    return ACE_OK;
}

int ace_prof_stop(double* total_ms, int32_t* launches) {
    g_err.clear();
    g_prof.on = false;
    for (int c = 0; c < ACE_NKCLASS; ++c) {
        if (total_ms) total_ms[c] = 0.0;
        if (launches) launches[c] = 0;
        g_prof.work_tot[c] = g_prof.bytes_tot[c] = g_prof.ops_tot[c] = 0.0;
    }
    for (size_t i = 0; i < g_prof.used; ++i) {
        ACE_HIP(hipEventSynchronize(g_prof.ev[2 * i + 1]));
        float ms = 0.f;
        ACE_HIP(hipEventElapsedTime(&ms, g_prof.ev[2 * i], g_prof.ev[2 * i + 1]));
        const int c = g_prof.cls[i];
        g_prof.work_tot[c] += g_prof.work[i];
        g_prof.bytes_tot[c] += g_prof.wbytes[i];
        g_prof.ops_tot[c] += g_prof.wops[i];
        if (total_ms) total_ms[c] += ms;
        if (launches) launches[c] += 1;
    }
    for (hipEvent_t e : g_prof.ev) (void)hipEventDestroy(e);
    g_prof.ev.clear();
    g_prof.cls.clear();
    g_prof.work.clear();
    g_prof.wbytes.clear();
    g_prof.wops.clear();
    g_prof.used = 0;
    ACE_HIP(hipDeviceSynchronize());   // (the m-space counters are copied after the last events)
    g_prof.msp_total = 0;
    for (int i = 0; i < g_prof.msp_used; ++i) g_prof.msp_total += g_prof.msp_slots[i];
    g_prof.msp_used = 0;
    return ACE_OK;
}

void ace_admm_cfg_default(ace_admm_cfg* c) {
    std::memset(c, 0, sizeof *c);
    c->variant = ACE_VARIANT_A2ONLY;
    c->scale_by_row = 1;
    c->use_rank_one = 0;
    c->maxiter = 500;
    c->fixed_iters = 0;
    c->a_shared = 1;
    c->eig_warm = 1;
    c->mu0 = 1e-3;
    c->rho = 1.03;
    c->tol_rel = 1e-4;
    c->tol_abs = 1e-8;
    c->r = 1;
    c->rank_one = nullptr;
}

size_t ace_admm_workspace_size(const ace_admm_cfg* cfg, int batch, int m, int n) {
    if (!cfg || batch < 1 || m < 1 || n < 1) return 0;
    Carver cv{nullptr};
    LinOps L;
    AdmmState w;
    linops_carve(cv, cfg->a_shared != 0, batch, m, n, &L);
    admm_state_carve(cv, batch, m, n, std::max(1, cols(cfg)), &w);
    return cv.off + 256;
}

}  // extern "C"

namespace {
int solve_core(const ace_admm_cfg* cfg, int batch, int m, int n, int tx, int rx, int prof_tx, int prof_n,
               const double* A, const double* B, const double* X0, double* Xo, double* Yo, int32_t* iters,
               uint32_t* status, double* mu_out, void* workspace, size_t workspace_bytes, hipStream_t st);

// A2only with an odd tx.  The reference reshapes z to tx x rx for any tx (inferLowRankV4_multi.m:426); the
// Z-prox's parallel Jacobi pairs rows, so the problem is solved as the (tx + 1) x rx one whose extra row is
// zero: A's columns tx + (tx + 1) j are zero, hence that row of X (= (I + A^H A)^{-1}(A^H T + Z - N / mu)), of
// E = X + N / mu, Z and N stays exactly zero (E E^H gets an exact zero eigenpair whose U^H E row is zero), and
// every other entry follows the tx x rx problem's arithmetic.  The rank profile keeps the original tx and n
// (:437-464).  The padded A, X0, X and workspace are this call's own allocations, released after the solve's
// stream drains (so this shape returns synchronously).
int solve_odd_tx(const ace_admm_cfg* cfg, int batch, int m, int n, int tx, int rx, const double* A,
                 const double* B, const double* X0, double* Xo, double* Yo, int32_t* iters, uint32_t* status,
                 double* mu_out, hipStream_t st) {
    const int txp = tx + 1, np = txp * rx, r = cols(cfg), R = cfg->scale_by_row ? r : 1;
    const size_t arows = (size_t)(cfg->a_shared ? 1 : batch) * m * rx, xrows = (size_t)batch * r * rx,
                 orows = (size_t)batch * R * rx, ws = ace_admm_workspace_size(cfg, batch, m, np) + 4096;
    void *dA = nullptr, *dX0 = nullptr, *dX = nullptr, *dW = nullptr;
    hipError_t e = hipMalloc(&dA, arows * txp * 16);
    if (e == hipSuccess) e = hipMalloc(&dX0, xrows * txp * 16);
    if (e == hipSuccess) e = hipMalloc(&dX, orows * txp * 16);
    if (e == hipSuccess) e = hipMalloc(&dW, ws);
    auto release = [&]() {   // (the solve's work on st must finish before its buffers go)
        (void)hipStreamSynchronize(st);
        for (void* q : {dA, dX0, dX, dW})
            if (q) (void)hipFree(q);
    };
    // [rows][tx] runs of complex entries -> [rows][tx + 1] with a zero last entry
    if (e == hipSuccess) e = hipMemsetAsync(dA, 0, arows * txp * 16, st);
    if (e == hipSuccess) e = hipMemsetAsync(dX0, 0, xrows * txp * 16, st);
    if (e == hipSuccess)
        e = hipMemcpy2DAsync(dA, (size_t)txp * 16, A, (size_t)tx * 16, (size_t)tx * 16, arows, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess)
        e = hipMemcpy2DAsync(dX0, (size_t)txp * 16, X0, (size_t)tx * 16, (size_t)tx * 16, xrows, hipMemcpyDeviceToDevice,
                             st);
    if (e != hipSuccess) {
        release();
        return fail(ACE_ERR_HIP, "odd-tx padding: %s", hipGetErrorString(e));
    }
    int rc = solve_core(cfg, batch, m, np, txp, rx, tx, n, (const double*)dA, B, (const double*)dX0, (double*)dX, Yo,
                        iters, status, mu_out, dW, ws, st);
    if (rc == ACE_OK &&
        (e = hipMemcpy2DAsync(Xo, (size_t)tx * 16, dX, (size_t)txp * 16, (size_t)tx * 16, orows, hipMemcpyDeviceToDevice,
                              st)) != hipSuccess)
        rc = fail(ACE_ERR_HIP, "odd-tx unpadding: %s", hipGetErrorString(e));
    const std::string keep = g_err;
    release();
    g_err = keep;
    return rc;
}
}  // namespace

extern "C" {

int ace_admm_solve_batch(const ace_admm_cfg* cfg, int batch, int m, int n, int tx, int rx, const double* A,
                         const double* B, const double* X0, double* Xo, double* Yo, int32_t* iters, uint32_t* status,
                         double* mu_out, void* workspace, size_t workspace_bytes, void* stream) {
    g_err.clear();
    int rc = validate(cfg, batch, m, n, tx, rx);
    if (rc) return rc;
    if (!A || !B || !X0 || !Xo || !Yo || !workspace) return fail(ACE_ERR_ARG, "NULL buffer");
    hipStream_t st = (hipStream_t)stream;
    if (cfg->variant == ACE_VARIANT_A2ONLY && (tx & 1))
        return solve_odd_tx(cfg, batch, m, n, tx, rx, A, B, X0, Xo, Yo, iters, status, mu_out, st);
    return solve_core(cfg, batch, m, n, tx, rx, 0, 0, A, B, X0, Xo, Yo, iters, status, mu_out, workspace,
                      workspace_bytes, st);
}

}  // extern "C"

namespace {
int solve_core(const ace_admm_cfg* cfg, int batch, int m, int n, int tx, int rx, int prof_tx, int prof_n,
               const double* A, const double* B, const double* X0, double* Xo, double* Yo, int32_t* iters,
               uint32_t* status, double* mu_out, void* workspace, size_t workspace_bytes, hipStream_t st) {
    const size_t need = ace_admm_workspace_size(cfg, batch, m, n);
    if (need > workspace_bytes)
        return fail(ACE_ERR_WORKSPACE, "workspace too small: need %zu bytes, got %zu", need, workspace_bytes);
    poison_workspace(workspace, workspace_bytes, st);
    Carver cv{(char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255)};
    LinOps L;
    AdmmState w;
    linops_carve(cv, cfg->a_shared != 0, batch, m, n, &L);
    admm_state_carve(cv, batch, m, n, cols(cfg), &w);
    L.A = A;
    L.allow_i8 = cfg->f64_applies == 0;
    ACE_TRY(linops_setup(L, batch, st));
    AdmmParams p{};
    p.variant = cfg->variant;
    p.r = cols(cfg);
    p.row_mode = cfg->scale_by_row != 0;
    p.maxiter = cfg->maxiter;
    p.fixed_iters = cfg->fixed_iters;
    p.eig_warm = cfg->eig_warm;
    p.mu0 = cfg->mu0;
    p.rho = cfg->rho;
    p.tol_rel = cfg->tol_rel;
    p.tol_abs = cfg->tol_abs;
    p.tx = tx;
    p.rx = rx;
    p.prof_tx = prof_tx;
    p.prof_n = prof_n;
    p.use_rank_one = cfg->use_rank_one;
    p.rank_one = cfg->rank_one;
    return admm_run(L, p, w, batch, B, X0, Xo, Yo, iters, status, mu_out, st);
}
}  // namespace

extern "C" {

int ace_admm_solve_host(const ace_admm_cfg* cfg, int batch, int m, int n, int tx, int rx, const double* A,
                        const double* B, const double* X0, double* X, double* Y, int32_t* iters, uint32_t* status,
                        double* mu) {
    g_err.clear();
    int rc = validate(cfg, batch, m, n, tx, rx);
    if (rc) return rc;
    const int r = cols(cfg), R = cfg->scale_by_row ? r : 1;
    const size_t nA = (size_t)(cfg->a_shared ? 1 : batch) * m * n * 16;
    const size_t nB = (size_t)batch * m * 8, nX0 = (size_t)batch * r * n * 16, nX = (size_t)batch * R * n * 16,
                 nY = (size_t)batch * R * m * 16;
    const size_t ws = ace_admm_workspace_size(cfg, batch, m, n) + 4096;
    std::vector<void*> bufs;
    auto dalloc = [&](size_t bytes, void** p) -> hipError_t {
        hipError_t e = hipMalloc(p, bytes);
        if (e == hipSuccess) bufs.push_back(*p);
        return e;
    };
    auto cleanup = [&]() {
        for (void* p : bufs) (void)hipFree(p);
        bufs.clear();
    };
    void *dA, *dB, *dX0, *dX, *dY, *dW, *dI, *dS, *dM, *dR = nullptr;
    hipError_t e = hipSuccess;
    if ((e = dalloc(nA, &dA)) || (e = dalloc(nB, &dB)) || (e = dalloc(nX0, &dX0)) || (e = dalloc(nX, &dX)) ||
        (e = dalloc(nY, &dY)) || (e = dalloc(ws, &dW)) || (e = dalloc(4 * (size_t)batch, &dI)) ||
        (e = dalloc(4 * (size_t)batch, &dS)) || (e = dalloc(8 * (size_t)batch, &dM)) ||
        (cfg->rank_one && (e = dalloc((size_t)batch, &dR)))) {
        cleanup();
        return fail(ACE_ERR_HIP, "hipMalloc: %s", hipGetErrorString(e));
    }
#define ACE_HIPC(call)                                                                               \
    do {                                                                                             \
        hipError_t e_ = (call);                                                                      \
        if (e_ != hipSuccess) {                                                                      \
            cleanup();                                                                               \
            return fail(ACE_ERR_HIP, "%s: %s", #call, hipGetErrorString(e_));                        \
        }                                                                                            \
    } while (0)
    ACE_HIPC(hipMemcpy(dA, A, nA, hipMemcpyHostToDevice));
    ACE_HIPC(hipMemcpy(dB, B, nB, hipMemcpyHostToDevice));
    ACE_HIPC(hipMemcpy(dX0, X0, nX0, hipMemcpyHostToDevice));
    ace_admm_cfg dcfg = *cfg;   // the per-realisation flags, if any, as a device array
    if (cfg->rank_one) {
        ACE_HIPC(hipMemcpy(dR, cfg->rank_one, (size_t)batch, hipMemcpyHostToDevice));
        dcfg.rank_one = (const uint8_t*)dR;
    }
    rc = ace_admm_solve_batch(&dcfg, batch, m, n, tx, rx, (const double*)dA, (const double*)dB, (const double*)dX0,
                              (double*)dX, (double*)dY, (int32_t*)dI, (uint32_t*)dS, (double*)dM, dW, ws, nullptr);
    if (rc) {
        std::string keep = g_err;
        cleanup();
        g_err = keep;
        return rc;
    }
    ACE_HIPC(hipDeviceSynchronize());
    ACE_HIPC(hipMemcpy(X, dX, nX, hipMemcpyDeviceToHost));
    ACE_HIPC(hipMemcpy(Y, dY, nY, hipMemcpyDeviceToHost));
    if (iters) ACE_HIPC(hipMemcpy(iters, dI, 4 * (size_t)batch, hipMemcpyDeviceToHost));
    if (status) ACE_HIPC(hipMemcpy(status, dS, 4 * (size_t)batch, hipMemcpyDeviceToHost));
    if (mu) ACE_HIPC(hipMemcpy(mu, dM, 8 * (size_t)batch, hipMemcpyDeviceToHost));
#undef ACE_HIPC
    cleanup();
    return ACE_OK;
}

int ace_nuclear_prox_batch(int batch, int n, int r, const double* E, double tau, double* Z, void* stream) {
    g_err.clear();
    if (!E || !Z) return fail(ACE_ERR_ARG, "NULL buffer");
    if (batch < 1 || n < 1 || r < 1) return fail(ACE_ERR_ARG, "batch/n/r must be >= 1 (got %d/%d/%d)", batch, n, r);
    if (r > 32 || n > 4096) return fail(ACE_ERR_UNSUPPORTED, "nuclear prox needs r <= 32 and n <= 4096 (got %d, %d)", r, n);
    if (!(tau > 0) || !std::isfinite(tau)) return fail(ACE_ERR_ARG, "tau must be finite and > 0");
    const int e = launch_nuclear_prox(batch, n, r, E, tau, Z, (hipStream_t)stream);
    if (e) return fail(ACE_ERR_HIP, "nuclear prox: %s", hipGetErrorString((hipError_t)e));
    return ACE_OK;
}

int ace_synth_codebook(uint64_t seed, int64_t first, int count, int m, int n, double* A, void* stream) {
    g_err.clear();
    if (!A || count < 1 || m < 1 || n < 1) return fail(ACE_ERR_ARG, "bad synth_codebook arguments");
    launch_synth_codebook(seed, first, count, m, n, A, (hipStream_t)stream);
    ACE_HIP(hipGetLastError());
    return ACE_OK;
}

int ace_synth_channels(uint64_t seed, int64_t first, int count, int m, int tx, int rx, int L, double snr_db,
                       double x0_noise, const double* A, int a_shared, double* vecH, double* B, double* X0,
                       void* stream) {
    g_err.clear();
    if (!A || !vecH || !B || !X0 || count < 1 || m < 1 || tx < 1 || rx < 1 || L < 1 || L > 64 || first < 0)
        return fail(ACE_ERR_ARG, "bad synth_channels arguments");
    launch_synth_channels(seed, first, count, m, tx, rx, L, snr_db, x0_noise, A, a_shared, vecH, B, X0,
                          (hipStream_t)stream);
    ACE_HIP(hipGetLastError());
    return ACE_OK;
}

}  // extern "C"
