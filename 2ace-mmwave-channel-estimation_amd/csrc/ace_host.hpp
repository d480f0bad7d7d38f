// Host-side helpers shared by the C-ABI translation units (ace_api.cpp, ace_admm.cpp,
// ace_pipeline.cpp): thread-local error text, HIP error checks, the event-pair kernel
// timer behind ace_prof_start/stop, and the ArgMinZ rank profile.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <string>
#include <vector>

#include "ace_common.hpp"

namespace ace {

inline thread_local std::string g_err;

__attribute__((format(printf, 2, 3))) inline int fail(int code, const char* fmt, ...) {
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

#define ACE_TRY(call)          \
    do {                       \
        int rc_ = (call);      \
        if (rc_) return rc_;   \
    } while (0)

// ---- event-pair kernel timing (ace_prof_start / ace_prof_stop)
struct Prof {
    bool on = false;
    std::vector<hipEvent_t> ev;   // 2 per record
    std::vector<int> cls;
    std::vector<double> work;     // algorithmic flops of each recorded launch (ProfScope)
    std::vector<double> wbytes;   // algorithmic HBM bytes of each recorded launch
    std::vector<double> wops;     // int8 matrix-core ops of each recorded launch
    double work_tot[ACE_NKCLASS] = {};   // per class, over the recorded launches (ace_prof_work)
    double bytes_tot[ACE_NKCLASS] = {};  // (ace_prof_work_ex)
    double ops_tot[ACE_NKCLASS] = {};
    size_t used = 0;
    int stride = 1;               // record every stride-th launch of each class (ace_prof_sample) ...
    unsigned full = 0;            // ... except the classes in this mask, recorded on every launch
    int seen[ACE_NKCLASS] = {};
    // m-space step counts of the solves in the session (ace_prof_msp_steps): one pinned slot per
    // solve, filled from the device counter (AdmmState::done[1]) at the end of the solve
    int* msp_slots = nullptr;
    int msp_cap = 0, msp_used = 0;
    long long msp_total = 0;
};
inline Prof g_prof;
// solves per apply path since the last reset (ace_path_counts): 0 shared phase code (int8 digit
// planes), 1 private phase codes (2-bit code images), 2 f64 shared A, 3 f64 private A
inline std::atomic<long long> g_path[4];

// Host <-> device copies of host (pageable) buffers ordered on `st` for any stream kind: through a
// per-thread pinned staging buffer, the device -> host direction followed by a stream
// synchronisation.  (Pageable-memory hipMemcpyAsync on a non-blocking stream was measured returning
// values the stream's earlier kernels had not written yet: the driver's concurrent sweep points.)
struct Pinned {
    void* p = nullptr;
    size_t cap = 0;
    ~Pinned() {
        if (p) (void)hipHostFree(p);
    }
    hipError_t reserve(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = bytes < 4096 ? 4096 : bytes;
        const hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    }
};
inline thread_local Pinned g_stage;
inline hipError_t read_back(void* dst, const void* src, size_t bytes, hipStream_t st) {
    hipError_t e = g_stage.reserve(bytes);
    if (e == hipSuccess) e = hipMemcpyAsync(g_stage.p, src, bytes, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) memcpy(dst, g_stage.p, bytes);
    return e;
}
inline hipError_t upload(void* dst, const void* src, size_t bytes, hipStream_t st) {
    hipError_t e = g_stage.reserve(bytes);
    if (e == hipSuccess) e = hipStreamSynchronize(st);   // (the staging buffer may still be in use)
    if (e == hipSuccess) memcpy(g_stage.p, src, bytes);
    if (e == hipSuccess) e = hipMemcpyAsync(dst, g_stage.p, bytes, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e;
}

// ACE_POISON=1 (debugging): fill a solve's workspace with 0xFF bytes (NaN doubles, -1 ints) before
// it is carved, so that a read of memory the solve did not write shows up in its results
inline void poison_workspace(void* ws, size_t bytes, hipStream_t st) {
    static const bool on = [] {
        const char* e = exp_env("ACE_POISON");
        return e && e[0] == '1';
    }();
    if (on) (void)hipMemsetAsync(ws, 0xFF, bytes, st);
}

struct ProfScope {  // brackets one launch (or a short sequence) of class `c` on stream `st`
    hipStream_t st;
    int idx = -1;
    // work: the launch's algorithmic flops (8 per complex MAC), bytes: its algorithmic HBM bytes (each
    // array read or written once), ops: its int8 matrix-core ops; 0 where the caller accounts itself
    ProfScope(int c, hipStream_t s, double work = 0.0, double bytes = 0.0, double ops = 0.0) : st(s) {
        const bool pick = ((g_prof.full >> c) & 1u) || (g_prof.seen[c] % g_prof.stride) == 0;
        if (g_prof.on) ++g_prof.seen[c];
        if (g_prof.on && pick && g_prof.used < g_prof.cls.size()) {
            idx = (int)g_prof.used++;
            g_prof.cls[idx] = c;
            g_prof.work[idx] = work;
            g_prof.wbytes[idx] = bytes;
            g_prof.wops[idx] = ops;
            (void)hipEventRecord(g_prof.ev[2 * idx], st);
        }
    }
    ~ProfScope() {
        if (idx >= 0) (void)hipEventRecord(g_prof.ev[2 * idx + 1], st);
    }
};

// ArgMinZ rank profile for use_rank_one = 0 / 1 (inferLowRankV4_multi.m:437-464).
inline int rank_profile(int tx, int rx, int m, int n, int use_rank_one, int* rl, double* fl) {
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

// Bump allocator over a caller-provided device workspace (256-B aligned chunks);
// with base == nullptr it only measures.
struct Carver {
    char* base;
    size_t off = 0;
    template <class T = double>
    T* take(size_t bytes) {
        char* p = base ? base + off : nullptr;
        off += (bytes + 255) & ~(size_t)255;
        return reinterpret_cast<T*>(p);
    }
};

// ---- one ADMM solve (InferADMM, inferLowRankV4_multi.m:281-386) over a batch -------
// The sensing operator of the solve.  Shared regime: one A (m x n) for the batch with
// its A^H; private regime: A_b per realisation (r = 1 only).  K = A A^H and
// G = (I + K)^{-1} ([1 | batch][m][m]) are built by admm_setup.
struct LinOps {
    bool shared;
    int m, n;
    const double* A;
    double* AH;
    double* K;
    double* G;
    double* ns;  // shared regime: Newton-Schulz scratch (4 m x m: I + K, I, R, X', then 2 doubles:
                 // max|R| and the Gershgorin bound), else null
    // shared regime, phase-code A (every real component in {0, +-c}): the int8 fragment images of
    // A and A^H for the exact digit-plane applies (ace_i8gemm.hip); i8ok is set by linops_setup
    int8_t* LA8;
    int8_t* LAH8;
    int8_t* LK8;  // the two base-128 digit planes of K / c^2
    double* c8;   // device: c, c^2
    int* i8flag;  // device: set when some component is not in {0, +-c}
    bool i8ok;
    double* Gf;     // G in f64 MFMA fragment order (m <= GYK_MAXM; built by linops_setup)
    double* Kfr;    // K in the same fragment order (the A2nuclear m-space iteration, ace_nucmsp.hip)
    bool frag_ok;   // Gf, Kfr hold G, K
    bool gyk_ok;
    bool allow_i8;  // caller's choice (ace_admm_cfg::f64_applies == 0), set before linops_setup
    // private regime, phase-code A_b (ace_private.hip): 2-bit code images, c_b, and G_b as lower
    // tiles in G (K holds the Gauss-Jordan workspace); pc_ok is set by linops_setup
    uint32_t* pcodes;
    double* pcb;
    int* pcflag;
    bool pc_ok;
    int batch;      // realisations of the private operators
};
size_t linops_bytes(bool shared, int batch, int m, int n);
void linops_carve(Carver& cv, bool shared, int batch, int m, int n, LinOps* L);
int linops_setup(LinOps& L, int batch, hipStream_t st);  // K, G, A^H from L.A

struct AdmmParams {
    int variant, r, row_mode, maxiter, fixed_iters, eig_warm;
    double mu0, rho, tol_rel, tol_abs;
    int tx, rx;
    int prof_tx, prof_n;               // the rank profile's tx and n when they differ from the layout's (odd tx,
                                       // solved zero-padded to tx + 1 rows: ace_api.cpp); 0: tx, n
    int use_rank_one;                  // batch-wide flag (ignored where rank_one is given)
    const unsigned char* rank_one;     // per-realisation use_rank_one (device, may be null)
    // per-realisation train partitions (r > 1 stages only): L is the full A's operators, the state is in
    // m-space with each realisation's test rows held at zero (PartRows, ace_common.hpp); null: none
    const PartRows* part;
};
// Per-iteration state of a batch of `batch` realisations with r columns each.
struct AdmmState {
    double *X, *Z, *N, *V, *optX, *Q;
    double *Z2, *N2;  // ping-pong partners of Z, N for the r = 1 wmode iteration ([batch][n])
    double* AX;       // r = 1 unit path: AX of the last Y-step ([batch][m], RealState::avok)
    double *Y[2], *KY[2], *M, *S, *T, *g, *optY;
    double* ypart;  // fused Y-step partials [batch][ceil(m/64)][5] (r = 1 iterations)
    RealState* st;
    int* done;
    double* zeros;  // [n] c128 zeros (N of realisations with RealState::nzero)
    double *Sg[2], *optS;  // r = 1 m-space steady state (RealState::msp): S ping-pong, opt_S ([batch][m])
};
void admm_state_carve(Carver& cv, int batch, int m, int n, int r, AdmmState* s);
// Runs init (:296-310), the iterations (:318-383) and returns the best-objective iterate
// (:384-385) in Xo [batch][row_mode ? r : 1][n], Yo [..][m].  iters/status/mu optional.
int admm_run(const LinOps& L, const AdmmParams& p, const AdmmState& s, int batch, const double* B,
             const double* X0, double* Xo, double* Yo, int32_t* iters, uint32_t* status, double* mu,
             hipStream_t st);

}  // namespace ace
