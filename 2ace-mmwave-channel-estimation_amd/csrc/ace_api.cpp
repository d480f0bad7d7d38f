// Host driver and C-ABI (include/ace.h) of the MI355X 2ACE ADMM hot path.
//
// ace_admm_solve_batch runs InferADMM (main/src/my_recovery_algorithms/ADMM_v2/
// inferLowRankV4_multi.m:281-386) for a batch of independent realisations:
//   setup   K = A A^H, G = (I + K)^{-1}          (replaces U = inv(A'A+I), :286-289)
//   init    :296-310
//   iterate :318-383, one kernel sequence per iteration:
//     pre    V = Z - N/mu, S = Y - M/mu
//     T = S - A V          (MFMA GEMM, shared A  | GEMV, private A)
//     g = G T
//     ystep  AX = S - g, ArgMinY, M update        (:326-337)
//     KY = K Y                                    (for ||A'Y||, ||A'(Y-Y0)||)
//     X = V + A^H g                               (ArgMinX, :325)
//     zstep  ArgMinZ, N update, residuals, stop test, best tracking, mu update
//   finalize opt_X / opt_Y (:384-385)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ace_common.hpp"

using namespace ace;

namespace {
thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define ACE_HIP(call)                                                                                  \
    do {                                                                                               \
        hipError_t e_ = (call);                                                                        \
        if (e_ != hipSuccess) return fail(ACE_ERR_HIP, "%s: %s (%s:%d)", #call, hipGetErrorString(e_), \
                                          __FILE__, __LINE__);                                         \
    } while (0)

// ArgMinZ rank profile (inferLowRankV4_multi.m:437-464)
int rank_profile(int tx, int rx, int m, int n, int use_rank_one, int* rl, double* fl) {
    const int sz = tx < rx ? tx : rx;
    const int r0 = (int)std::ceil(std::sqrt((double)sz) * 0.5), r1 = (int)std::ceil(std::sqrt((double)sz) * 0.7);
    const int r2 = (int)std::ceil(std::sqrt((double)sz));
    int r3 = (int)std::ceil(std::sqrt((double)sz) * 2.0);
    if (r3 > sz) r3 = sz;
    if (use_rank_one) { rl[0] = 1; fl[0] = 0.95; return 1; }
    if (m >= n * 3) { rl[0] = r3; fl[0] = 0.995; return 1; }
    if (r1 <= 2) { rl[0] = r2; fl[0] = 0.95; return 1; }
    if (r0 <= 2) {
        rl[0] = r1; rl[1] = r2; rl[2] = r3;
        fl[0] = 0.9; fl[1] = 0.95; fl[2] = 0.995;
        return 3;
    }
    rl[0] = r0; rl[1] = r1; rl[2] = r2; rl[3] = r3;
    fl[0] = 0.8; fl[1] = 0.9; fl[2] = 0.95; fl[3] = 0.995;
    return 4;
}

// Workspace carve-up (all chunks 256-B aligned).
struct Ws {
    double *AH, *K, *G;                      // shared: AH n x m; K, G: [mats][m][m]
    double *X, *Z, *N, *V, *optX, *Q;        // [batch][n], Q [batch][tx*tx]
    double *Y[2], *KY[2], *M, *S, *T, *g, *optY;  // [batch][m]
    RealState* st;
    int* done;
    size_t bytes;
};

size_t carve(const ace_admm_cfg* c, int batch, int m, int n, int tx, char* base, Ws* w) {
    size_t off = 0;
    auto take = [&](size_t bytes) -> char* {
        char* p = base ? base + off : nullptr;
        off += (bytes + 255) & ~(size_t)255;
        return p;
    };
    const size_t cz = 16;
    const size_t mats = c->a_shared ? 1 : (size_t)batch;
    w->AH = c->a_shared ? (double*)take(cz * n * m) : nullptr;
    w->K = (double*)take(cz * mats * m * m);
    w->G = (double*)take(cz * mats * m * m);
    w->X = (double*)take(cz * batch * n);
    w->Z = (double*)take(cz * batch * n);
    w->N = (double*)take(cz * batch * n);
    w->V = (double*)take(cz * batch * n);
    w->optX = (double*)take(cz * batch * n);
    w->Q = (c->variant == ACE_VARIANT_A2ONLY) ? (double*)take(cz * batch * tx * tx) : nullptr;
    for (int i = 0; i < 2; ++i) w->Y[i] = (double*)take(cz * batch * m);
    for (int i = 0; i < 2; ++i) w->KY[i] = (double*)take(cz * batch * m);
    w->M = (double*)take(cz * batch * m);
    w->S = (double*)take(cz * batch * m);
    w->T = (double*)take(cz * batch * m);
    w->g = (double*)take(cz * batch * m);
    w->optY = (double*)take(cz * batch * m);
    w->st = (RealState*)take(sizeof(RealState) * batch);
    w->done = (int*)take(256);
    w->bytes = off;
    return off;
}

// ---- event-pair kernel timing (ace_prof_start / ace_prof_stop)
struct Prof {
    bool on = false;
    std::vector<hipEvent_t> ev;   // 2 per record
    std::vector<int> cls;
    size_t used = 0;
} g_prof;

struct ProfScope {  // brackets one launch (or a short sequence) of class `c` on stream `st`
    hipStream_t st;
    int idx = -1;
    ProfScope(int c, hipStream_t s) : st(s) {
        if (g_prof.on && g_prof.used < g_prof.cls.size()) {
            idx = (int)g_prof.used++;
            g_prof.cls[idx] = c;
            (void)hipEventRecord(g_prof.ev[2 * idx], st);
        }
    }
    ~ProfScope() {
        if (idx >= 0) (void)hipEventRecord(g_prof.ev[2 * idx + 1], st);
    }
};

int validate(const ace_admm_cfg* c, int batch, int m, int n, int tx, int rx) {
    if (!c) return fail(ACE_ERR_ARG, "cfg is NULL");
    if (batch < 1 || m < 1 || n < 1) return fail(ACE_ERR_ARG, "batch/m/n must be >= 1 (got %d/%d/%d)", batch, m, n);
    if (tx * rx != n) return fail(ACE_ERR_ARG, "n (%d) != tx*rx (%d*%d)", n, tx, rx);
    if (c->variant != ACE_VARIANT_A2ONLY && c->variant != ACE_VARIANT_NUCLEAR)
        return fail(ACE_ERR_ARG, "unknown variant %d", c->variant);
    if (c->variant == ACE_VARIANT_A2ONLY && (tx < 2 || tx > 32 || (tx & 1) || rx > 32))
        return fail(ACE_ERR_UNSUPPORTED, "A2only Z-prox needs even tx in [2,32] and rx <= 32 (got %d, %d)", tx, rx);
    if (n > 4096 || m > 4096) return fail(ACE_ERR_UNSUPPORTED, "m, n must be <= 4096 (got %d, %d)", m, n);
    if (c->maxiter < 1) return fail(ACE_ERR_ARG, "maxiter must be >= 1");
    if (!(c->mu0 > 0) || !(c->rho > 0)) return fail(ACE_ERR_ARG, "mu0 and rho must be > 0");
    return ACE_OK;
}
}  // namespace

extern "C" {

const char* ace_last_error(void) { return g_err.c_str(); }
const char* ace_version(void) { return "ace-mi355x 0.1.0 (gfx950)"; }

int ace_prof_start(int max_launches) {
    g_err.clear();
    if (max_launches < 1) return fail(ACE_ERR_ARG, "max_launches must be >= 1");
    for (hipEvent_t e : g_prof.ev) (void)hipEventDestroy(e);
    g_prof.ev.assign(2 * (size_t)max_launches, nullptr);
    for (auto& e : g_prof.ev) ACE_HIP(hipEventCreate(&e));
    g_prof.cls.assign(max_launches, 0);
    g_prof.used = 0;
    g_prof.on = true;
    return ACE_OK;
}

int ace_prof_stop(double* total_ms, int32_t* launches) {
    g_err.clear();
    g_prof.on = false;
    for (int c = 0; c < ACE_NKCLASS; ++c) {
        if (total_ms) total_ms[c] = 0.0;
        if (launches) launches[c] = 0;
    }
    for (size_t i = 0; i < g_prof.used; ++i) {
        ACE_HIP(hipEventSynchronize(g_prof.ev[2 * i + 1]));
        float ms = 0.f;
        ACE_HIP(hipEventElapsedTime(&ms, g_prof.ev[2 * i], g_prof.ev[2 * i + 1]));
        const int c = g_prof.cls[i];
        if (total_ms) total_ms[c] += ms;
        if (launches) launches[c] += 1;
    }
    for (hipEvent_t e : g_prof.ev) (void)hipEventDestroy(e);
    g_prof.ev.clear();
    g_prof.cls.clear();
    g_prof.used = 0;
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
}

size_t ace_admm_workspace_size(const ace_admm_cfg* cfg, int batch, int m, int n) {
    if (!cfg || batch < 1 || m < 1 || n < 1) return 0;
    Ws w;  // Q is sized for the largest supported tx (32)
    return carve(cfg, batch, m, n, 32, nullptr, &w) + 256;
}

int ace_admm_solve_batch(const ace_admm_cfg* cfg, int batch, int m, int n, int tx, int rx, const double* A,
                         const double* B, const double* X0, double* Xo, double* Yo, int32_t* iters, uint32_t* status,
                         double* mu_out, void* workspace, size_t workspace_bytes, void* stream) {
    g_err.clear();
    int rc = validate(cfg, batch, m, n, tx, rx);
    if (rc) return rc;
    if (!A || !B || !X0 || !Xo || !Yo || !workspace) return fail(ACE_ERR_ARG, "NULL buffer");
    hipStream_t st = (hipStream_t)stream;
    Ws w;
    char* base = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
    const size_t need = carve(cfg, batch, m, n, 32, nullptr, &w) + (size_t)(base - (char*)workspace);
    if (need > workspace_bytes)
        return fail(ACE_ERR_WORKSPACE, "workspace too small: need %zu bytes, got %zu", need, workspace_bytes);
    carve(cfg, batch, m, n, 32, base, &w);
    const bool shared = cfg->a_shared != 0;
    const long long mm = (long long)m * m, mn = (long long)m * n;

    // ---- setup: K = A A^H, G = (I + K)^{-1}, A^H (shared regime)
    const int mats = shared ? 1 : batch;
    {
    ProfScope ps(ACE_K_SETUP, st);
    // K[j][i] = sum_k conj(A[i][k]) A[j][k]  : GEMM with L = conj(A), V = rows of A
    launch_zgemm(0, true, m, n, m, A, n, mn, A, n, mn, w.K, nullptr, m, mm, mats, st);
    ACE_HIP(hipMemcpyAsync(w.G, w.K, sizeof(double) * 2 * mm * mats, hipMemcpyDeviceToDevice, st));
    launch_inv_ipk(m, mats, w.G, mm, st);
    if (shared) launch_conj_transpose(m, n, A, w.AH, st);
    }
    ACE_HIP(hipGetLastError());

    auto applyA = [&](int mode, const double* Vin, double* C, const double* E) {  // C = E (-) A Vin
        if (shared) launch_zgemm(mode, false, m, n, batch, A, n, 0, Vin, n, 0, C, E, m, 0, 1, st);
        else launch_zgemv_rows(mode, m, n, batch, A, mn, Vin, n, C, E, m, st);
    };
    auto applyMM = [&](const double* Lm, const double* Vin, double* C) {  // C = L Vin, L = G or K
        if (shared) launch_zgemm(0, false, m, m, batch, Lm, m, 0, Vin, m, 0, C, nullptr, m, 0, 1, st);
        else launch_zgemv_rows(0, m, m, batch, Lm, mm, Vin, m, C, nullptr, m, st);
    };
    auto applyAH = [&](const double* gin, double* C, const double* E) {  // C = E + A^H gin
        if (shared) launch_zgemm(2, false, n, m, batch, w.AH, m, 0, gin, m, 0, C, E, n, 0, 1, st);
        else launch_zgemv_cols(2, m, n, batch, A, mn, gin, m, C, E, n, st);
    };

    ZArgs za{};
    za.n = n;
    za.m = m;
    za.tx = tx;
    za.rx = rx;
    za.X = w.X;
    za.N = w.N;
    za.Z = w.Z;
    za.Q = w.Q;
    za.st = w.st;
    za.optX = w.optX;
    za.optY = w.optY;
    za.done_count = w.done;
    za.np = rank_profile(tx, rx, m, n, cfg->use_rank_one, za.rl, za.fl);
    za.tol_rel = cfg->tol_rel;
    za.tol_abs = cfg->tol_abs;
    za.rho = cfg->rho;
    za.fixed_iters = cfg->fixed_iters;
    za.warm = cfg->eig_warm;

    // ---- init (:296-310)
    ACE_HIP(hipMemsetAsync(w.done, 0, 256, st));
    {
        ProfScope ps(ACE_K_INIT, st);
        applyA(0, X0, w.T, nullptr);                             // AX = A*X0
        launch_init(n, m, batch, X0, w.T, B, w.X, w.Y[0], w.M, w.N, w.st, cfg->mu0, st);
        za.it = 0;
        launch_zstep(cfg->variant, true, za, batch, st);         // Z = ArgMinZ(X, N=0, mu=1)
        applyMM(w.K, w.Y[0], w.KY[0]);                           // K*Y (for A'*Y terms)
    }
    ACE_HIP(hipGetLastError());

    int p = 0;
    const int poll = 8;
    for (int it = 1; it <= cfg->maxiter; ++it) {
        { ProfScope ps(ACE_K_PRE, st); launch_pre(n, m, batch, w.Z, w.N, w.Y[p], w.M, w.V, w.S, w.st, st); }
        { ProfScope ps(ACE_K_APPLY_A, st); applyA(1, w.V, w.T, w.S); }          // T = S - A V
        { ProfScope ps(ACE_K_APPLY_G, st); applyMM(w.G, w.T, w.g); }            // g = G T
        { ProfScope ps(ACE_K_YSTEP, st); launch_ystep(m, batch, w.S, w.g, w.M, B, w.Y[p], w.Y[1 - p], w.st, st); }
        { ProfScope ps(ACE_K_APPLY_K, st); applyMM(w.K, w.Y[1 - p], w.KY[1 - p]); }  // K Y
        { ProfScope ps(ACE_K_APPLY_AH, st); applyAH(w.g, w.X, w.V); }           // X = V + A^H g
        za.it = it;
        za.Ynew = w.Y[1 - p];
        za.Yold = w.Y[p];
        za.KYnew = w.KY[1 - p];
        za.KYold = w.KY[p];
        { ProfScope ps(ACE_K_ZSTEP, st); launch_zstep(cfg->variant, false, za, batch, st); }
        p = 1 - p;
        if (!cfg->fixed_iters && (it % poll == 0) && it < cfg->maxiter) {
            int h_done = 0;
            ACE_HIP(hipMemcpyAsync(&h_done, w.done, sizeof(int), hipMemcpyDeviceToHost, st));
            ACE_HIP(hipStreamSynchronize(st));
            if (h_done >= batch) break;
        }
    }
    ACE_HIP(hipGetLastError());
    {
        ProfScope ps(ACE_K_FINAL, st);
        launch_finalize(n, m, batch, w.optX, w.optY, w.X, w.Y[p], Xo, Yo, iters, status, mu_out, w.st, st);
    }
    ACE_HIP(hipGetLastError());
    return ACE_OK;
}

int ace_admm_solve_host(const ace_admm_cfg* cfg, int batch, int m, int n, int tx, int rx, const double* A,
                        const double* B, const double* X0, double* X, double* Y, int32_t* iters, uint32_t* status,
                        double* mu) {
    g_err.clear();
    int rc = validate(cfg, batch, m, n, tx, rx);
    if (rc) return rc;
    const size_t nA = (size_t)(cfg->a_shared ? 1 : batch) * m * n * 16;
    const size_t nB = (size_t)batch * m * 8, nX = (size_t)batch * n * 16, nY = (size_t)batch * m * 16;
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
    void *dA, *dB, *dX0, *dX, *dY, *dW, *dI, *dS, *dM;
    hipError_t e = hipSuccess;
    if ((e = dalloc(nA, &dA)) || (e = dalloc(nB, &dB)) || (e = dalloc(nX, &dX0)) || (e = dalloc(nX, &dX)) ||
        (e = dalloc(nY, &dY)) || (e = dalloc(ws, &dW)) || (e = dalloc(4 * (size_t)batch, &dI)) ||
        (e = dalloc(4 * (size_t)batch, &dS)) || (e = dalloc(8 * (size_t)batch, &dM))) {
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
    ACE_HIPC(hipMemcpy(dX0, X0, nX, hipMemcpyHostToDevice));
    rc = ace_admm_solve_batch(cfg, batch, m, n, tx, rx, (const double*)dA, (const double*)dB, (const double*)dX0,
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
