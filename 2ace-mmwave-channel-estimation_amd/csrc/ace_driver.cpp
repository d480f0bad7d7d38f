// Driver-level boundary: the MATLAB functions main.py calls through the MATLAB Engine,
//   [H_amp, H_angle] = channel_recovery_ADMM_v2_simulation_<A2only|A2nuclear|multiresolution|phaselift>(
//                          tx_ant_num, rx_ant_num, cb_amp, cb_angle, rss_final, seed_id)
// (main/channel_recovery_ADMM_v2_simulation_A2only.m:9-179, ..._A2nuclear.m,
//  ..._multiresolution.m; call sites main/main.py:308, :427-437).
//
// Per sweep point M (:106-118, 8 points up to 4*tx*rx):
//   M_idx = randperm(P, M)                          (:137; multiresolution: tiered, :137-144)
//   cb_train = cb(M_idx,:), rss_train = sqrt(db2pow(rss)/1000) * rss_fct   (:120, :132, :139)
//   picked_beams = 1:M (Random_Phase_State, Generate_Sensing_Matrix_with_candidate.m:13)
//   X = ADMM_v2(rss_train, cb_train, tx, rx, 4) = inferLowRankV4_multi / inferLowRank_Nuclear
//       (Recover_Channel.m:27-31, ADMM_v2.m:30-32)  -> ace_pipeline_solve_batch on the GPU
//   phaselift: X = MyPhaseLift((rss_train/2e5).^2*1e10, cb_train)/sqrt(1e10)*2e5
//       (Recover_Channel.m:32-35)                   -> ace_phaselift_solve_batch on the GPU
//   H_out(i,1,:) = X / rss_fct, NaN -> 0, H_amp = abs, H_angle = angle  (:170-178)
// The drivers' Generate_Channel / Sparse_Channel_Formulation calls (:146-149) feed only the
// baseline methods (their outputs never reach the ADMM recovery) and are not performed.
// RNG: MATLAB's rng/randperm/randsample streams cannot be reproduced outside MATLAB; the
// build draws the same distributions from its counter-based generator seeded by the
// reference's seed list (:103), so a given (seed_id, inputs) is reproducible here.
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ace_host.hpp"

using namespace ace;

namespace {

constexpr double kRssFct = 1e5 / 3.0;   // :125 rss_fct
const uint64_t kSeeds[40] = {58659179, 42737934, 36326041, 89830260, 90710947, 96474890, 33424536, 67991541,
                             42149446, 38961924, 54659060, 32629256, 33087755, 27433950, 9404442,  20146383,
                             84040563, 75325961, 47726929, 13999319, 5597853,  74801351, 37024073, 75534492,
                             99245881, 19650488, 5314224,  98859252, 60803022, 76056701, 14112116, 64027813,
                             73073690, 6288587,  42217659, 45632040, 7495955,  31960297, 92863244, 93081516};
const uint64_t kNuclearSeeds[4] = {1024, 2048, 4096, 8192};   // ..._A2nuclear.m:103

// multiresolution tiers (..._multiresolution.m:111-112, :137-144): for 16 antennas rows
// [0, 1984) are the 4-antenna-group probes, then 3968 2-antenna-group probes, then 3968
// per-antenna probes, picked by M <= 96 / <= 256 / else.  The reference defines tiers for 16
// antennas only; the 32-antenna layout is the build's analogue (ace_amd.synth.multires_tiers:
// 4x the rows and 4x the thresholds).
const int kTierLen16[3] = {1984, 3968, 3968}, kThresh16[2] = {96, 256};
const int kTierLen32[3] = {7936, 15872, 15872}, kThresh32[2] = {384, 1024};
bool multires_defined(int tx, int rx) { return tx == rx && (tx == 16 || tx == 32); }
int multires_tier(int M, int tx) {
    const int* th = tx == 32 ? kThresh32 : kThresh16;
    return M <= th[0] ? 0 : (M <= th[1] ? 1 : 2);
}
int tier_len(int tx, int t) { return (tx == 32 ? kTierLen32 : kTierLen16)[t]; }

// splitmix64 counter RNG (the same construction as ace_synth.hip / ace_amd.synth)
uint64_t sm64(uint64_t seed, uint64_t stream, uint64_t ctr) {
    uint64_t z = (seed ^ (stream * 0xD1B54A32D192ED03ull)) + (ctr + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// first k entries of a uniformly random permutation of 0..P-1 (partial Fisher-Yates):
// randperm(P, k) / randsample(P, k) without replacement, 0-based, in sampled order
void randperm_k(uint64_t seed, uint64_t stream, int P, int k, int32_t* out) {
    std::vector<int32_t> p(P);
    for (int i = 0; i < P; ++i) p[i] = i;
    for (int i = 0; i < k; ++i) {
        const uint64_t u = sm64(seed, stream, (uint64_t)i) >> 11;                 // 53 bits
        const int j = i + (int)(((double)u * (1.0 / 9007199254740992.0)) * (P - i));
        std::swap(p[i], p[std::min(j, P - 1)]);
        out[i] = p[i];
    }
}

// M sweep (:106-118): round(linspace(2, sqrt(4*tx*rx), 8)).^2 for 4/8/16/32/36 antennas
int m_sweep(int tx, int rx, int32_t* M) {
    const auto ok = [](int a) { return a == 4 || a == 8 || a == 16 || a == 32 || a == 36; };
    if (!ok(tx) && !ok(rx)) return 0;
    const double hi = std::sqrt(4.0 * tx * rx);
    for (int i = 0; i < 8; ++i) {
        const double v = 2.0 + (hi - 2.0) * i / 7.0;
        const double r = std::round(i == 7 ? hi : v);   // linspace hits the end point exactly
        M[i] = (int32_t)(r * r);
    }
    return 8;
}


// exp(1j*angle) with the components MATLAB's phase-code angles leave a rounding residue in
// (cos(pi/2) = 6.1e-17, sin(pi) = 1.2e-16) snapped to the exact 0 / +-1 they stand for: within
// 4 ulp of 1 for |value| ~ 1 and 1e-15 for |value| ~ 0, i.e. a change below 1e-15 of the amplitude.
// A phase-code codebook passed as |cb| / angle(cb) (main.py:301-302) is then the exact phase
// code again, whose applies run as int8 digit planes; any other codebook moves
// by less than the rounding of its own cos / sin.
inline double snap_unit(double v) {
    if (std::fabs(v) < 1e-15) return 0.0;
    if (std::fabs(std::fabs(v) - 1.0) <= 4 * 2.220446049250313e-16) return std::copysign(1.0, v);
    return v;
}

// A resident device buffer set for one sweep point, released on every exit path.
struct DevBufs {
    std::vector<void*> p;
    hipStream_t st = nullptr;
    hipError_t alloc(size_t bytes, void** q) {
        hipError_t e = hipMalloc(q, bytes);
        if (e == hipSuccess) p.push_back(*q);
        return e;
    }
    ~DevBufs() {
        if (st) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
        for (void* q : p) (void)hipFree(q);
    }
};

// One sweep point i (M rows): rows, cb_train / rss_train, the solve, H row (:137-178).
int sweep_point(int driver, int tx, int rx, int P, const double* cb_amp, const double* cb_angle,
                const double* rss_dbm, uint64_t seed, int i, int M, int dev, int maxiter, double* H_amp,
                double* H_angle) {
    g_err.clear();
    ACE_HIP(hipSetDevice(dev));
    const int n = tx * rx;
    ace_pipeline_cfg cfg;
    ace_pipeline_cfg_default(&cfg, driver == ACE_DRIVER_A2NUCLEAR ? ACE_VARIANT_NUCLEAR : ACE_VARIANT_A2ONLY);
    if (maxiter > 0) cfg.maxiter = maxiter;
    // ---- :137 M_idx = randperm(length(rss_final), M) (multiresolution: within its tier)
    std::vector<int32_t> idx(M);
    int avail = P, off = 0;
    if (driver == ACE_DRIVER_MULTIRES) {
        const int t = multires_tier(M, tx);
        avail = tier_len(tx, t);
        for (int k = 0; k < t; ++k) off += tier_len(tx, k);
    }
    randperm_k(seed, 0x100 + 2 * (uint64_t)i, avail, M, idx.data());
    // ---- :120, :138-139 cb_train (row-major M x n c128), rss_train
    std::vector<double> A(2 * (size_t)M * n), B(M);
    for (int r = 0; r < M; ++r) {
        const int row = idx[r] + off;
        for (int k = 0; k < n; ++k) {
            const double a = cb_amp[(size_t)row * n + k], ph = cb_angle[(size_t)row * n + k];
            A[2 * ((size_t)r * n + k)] = a * snap_unit(std::cos(ph));
            A[2 * ((size_t)r * n + k) + 1] = a * snap_unit(std::sin(ph));
        }
        B[r] = std::sqrt(std::pow(10.0, rss_dbm[row] / 10.0) / 1000.0) * kRssFct;   // db2pow
    }
    std::vector<double> X(2 * (size_t)n);
    if (driver != ACE_DRIVER_PHASELIFT) {
        const int r = std::min(std::min(cfg.r, M), n);
        const int mt = (int)std::floor(M * cfg.cc_frac);
        if (mt < r) {
            // ill-posed sweep point (fewer train rows than spectral columns, e.g. M = 4):
            // reported as NaN -> 0 like a failed MATLAB recovery (H_out(isnan) = 0, :176)
            for (int k = 0; k < n; ++k) H_amp[k] = H_angle[k] = 0.0;
            return ACE_OK;
        }
    }
    DevBufs d;
    ACE_HIP(hipStreamCreateWithFlags(&d.st, hipStreamNonBlocking));
    void *dA, *dB, *dX, *dY, *dW;
    const size_t nA = 16 * (size_t)M * n, nB = 8 * (size_t)M, nX = 16 * (size_t)n, nY = 16 * (size_t)M;
    if (driver == ACE_DRIVER_PHASELIFT) {
        // ---- Recover_Channel.m:32-35: MyPhaseLift((meas/2e5).^2*1e10, beams)/sqrt(1e10)*2e5
        ace_phaselift_cfg pcfg;
        ace_phaselift_cfg_default(&pcfg);
        if (maxiter > 0) pcfg.maxIts = maxiter;
        for (int r = 0; r < M; ++r) B[r] = (B[r] / 2e5) * (B[r] / 2e5) * 1e10;
        const size_t ws = ace_phaselift_workspace_size(&pcfg, 1, M, n);
        if (!ws) return fail(ACE_ERR_UNSUPPORTED, "phaselift: unsupported size M = %d, n = %d", M, n);
        ACE_HIP(d.alloc(nA, &dA));
        ACE_HIP(d.alloc(nB, &dB));
        ACE_HIP(d.alloc(nX, &dX));
        ACE_HIP(d.alloc(ws, &dW));
        ACE_HIP(upload(dA, A.data(), nA, d.st));
        ACE_HIP(upload(dB, B.data(), nB, d.st));
        ACE_TRY(ace_phaselift_solve_batch(&pcfg, 1, M, n, (const double*)dA, (const double*)dB, (double*)dX, nullptr,
                                          nullptr, dW, ws, d.st));
        ACE_HIP(read_back(X.data(), dX, nX, d.st));
        for (int k = 0; k < 2 * n; ++k) X[k] = X[k] / std::sqrt(1e10) * 2e5;
    } else {
        // ---- Recover_Channel -> ADMM_v2(..., 4): the pipeline with its own train partitions
        const int mt = (int)std::floor(M * cfg.cc_frac);
        std::vector<int32_t> tr((size_t)cfg.restarts * mt);
        for (int s = 0; s < cfg.restarts; ++s)
            randperm_k(seed, 0x101 + 2 * (uint64_t)i + 0x10000 * (uint64_t)s, M, mt, tr.data() + (size_t)s * mt);
        const size_t ws = ace_pipeline_workspace_size(&cfg, 1, M, n);
        if (!ws) return fail(ACE_ERR_UNSUPPORTED, "pipeline: unsupported size M = %d, n = %d", M, n);
        ACE_HIP(d.alloc(nA, &dA));
        ACE_HIP(d.alloc(nB, &dB));
        ACE_HIP(d.alloc(nX, &dX));
        ACE_HIP(d.alloc(nY, &dY));
        ACE_HIP(d.alloc(ws, &dW));
        ACE_HIP(upload(dA, A.data(), nA, d.st));
        ACE_HIP(upload(dB, B.data(), nB, d.st));
        ACE_TRY(ace_pipeline_solve_batch(&cfg, 1, M, n, tx, rx, (const double*)dA, (const double*)dB, tr.data(),
                                         (double*)dX, (double*)dY, nullptr, nullptr, nullptr, dW, ws, d.st));
        ACE_HIP(read_back(X.data(), dX, nX, d.st));
    }
    // ---- :170-178 H_out = X / rss_fct, NaN -> 0, amplitude and angle
    for (int k = 0; k < n; ++k) {
        std::complex<double> h(X[2 * k] / kRssFct, X[2 * k + 1] / kRssFct);
        if (std::isnan(h.real()) || std::isnan(h.imag())) h = 0.0;
        H_amp[k] = std::abs(h);
        H_angle[k] = std::arg(h);
    }
    return ACE_OK;
}

}  // namespace

extern "C" {

int ace_driver_m_sweep(int tx, int rx, int32_t* M_out) {
    g_err.clear();
    if (!M_out) return fail(ACE_ERR_ARG, "NULL M_out");
    const int k = m_sweep(tx, rx, M_out);
    if (!k) return fail(ACE_ERR_ARG, "Number of antenna on Tx and Rx must be 4/8/16/32! (got %d, %d)", tx, rx);
    return k;
}

int ace_driver_randperm(uint64_t seed, uint64_t stream, int P, int k, int32_t* out) {
    g_err.clear();
    if (!out || P < 1 || k < 0 || k > P) return fail(ACE_ERR_ARG, "randperm: need 0 <= k <= P (got P=%d k=%d)", P, k);
    randperm_k(seed, stream, P, k, out);
    return ACE_OK;
}

int ace_recover_driver(int driver, int tx, int rx, int P, const double* cb_amp, const double* cb_angle,
                       const double* rss_dbm, int seed_id, int n_M, const int32_t* M_list, double* H_amp,
                       double* H_angle) {
    return ace_recover_driver_ex(driver, tx, rx, P, cb_amp, cb_angle, rss_dbm, seed_id, n_M, M_list, 0, H_amp,
                                 H_angle);
}

int ace_recover_driver_ex(int driver, int tx, int rx, int P, const double* cb_amp, const double* cb_angle,
                          const double* rss_dbm, int seed_id, int n_M, const int32_t* M_list, int maxiter,
                          double* H_amp, double* H_angle) {
    g_err.clear();
    if (driver != ACE_DRIVER_A2ONLY && driver != ACE_DRIVER_A2NUCLEAR && driver != ACE_DRIVER_MULTIRES &&
        driver != ACE_DRIVER_PHASELIFT)
        return fail(ACE_ERR_ARG, "unknown driver %d", driver);
    if (!cb_amp || !cb_angle || !rss_dbm || !H_amp || !H_angle) return fail(ACE_ERR_ARG, "NULL buffer");
    if (tx < 1 || rx < 1 || P < 1) return fail(ACE_ERR_ARG, "tx, rx, P must be >= 1");
    if (seed_id < 1 || seed_id > 40) return fail(ACE_ERR_ARG, "seed_id must be in 1..40 (MATLAB seeds(seed_id))");
    int32_t sweep[8];
    std::vector<int32_t> Ms;
    if (M_list) {
        if (n_M < 1) return fail(ACE_ERR_ARG, "n_M must be >= 1");
        Ms.assign(M_list, M_list + n_M);
    } else {
        const int k = m_sweep(tx, rx, sweep);
        if (!k) return fail(ACE_ERR_ARG, "Number of antenna on Tx and Rx must be 4/8/16/32! (got %d, %d)", tx, rx);
        Ms.assign(sweep, sweep + k);
        n_M = k;
    }
    const int n = tx * rx;
    if (driver == ACE_DRIVER_MULTIRES && !multires_defined(tx, rx))
        return fail(ACE_ERR_UNSUPPORTED, "multiresolution tiers are defined for 16 x 16 (reference) and 32 x 32 "
                    "antennas (got %d x %d)", tx, rx);
    for (int i = 0; i < n_M; ++i) {
        const int M = Ms[i];
        int avail = P;
        if (driver == ACE_DRIVER_MULTIRES) {
            const int t = multires_tier(M, tx);
            avail = tier_len(tx, t);
            int off = 0;
            for (int k = 0; k < t; ++k) off += tier_len(tx, k);
            if (off + avail > P)
                return fail(ACE_ERR_ARG, "multiresolution codebook needs %d rows (tier %d), got %d", off + avail, t, P);
        }
        if (M < 1 || M > avail) return fail(ACE_ERR_ARG, "M = %d must be in [1, %d]", M, avail);
    }
    // seeds: A2only / multiresolution rng(seeds(seed_id)) (:103-104); A2nuclear rng(seeds(randi(4)))
    // (the build picks by seed_id); phaselift rng(4096) whatever seed_id (..._phaselift.m:127)
    const uint64_t seed = driver == ACE_DRIVER_A2NUCLEAR   ? kNuclearSeeds[(seed_id - 1) % 4]
                          : driver == ACE_DRIVER_PHASELIFT ? 4096
                                                           : kSeeds[seed_id - 1];

    // The sweep points are independent recoveries of different sizes M: each runs on its own host
    // thread, HIP stream and device buffers, so the 8 pipelines (whose restarts each synchronise
    // their stream once, ace_pipeline.cpp) overlap on the GPU; the call returns when all are done.
    int dev = 0;
    ACE_HIP(hipGetDevice(&dev));
    std::vector<int> rcs(n_M, ACE_OK);
    std::vector<std::string> errs(n_M);
    auto point = [&](int i) {
        rcs[i] = sweep_point(driver, tx, rx, P, cb_amp, cb_angle, rss_dbm, seed, i, Ms[i], dev, maxiter,
                             H_amp + (size_t)i * n, H_angle + (size_t)i * n);
        if (rcs[i]) errs[i] = g_err;
    };
    // ACE_DRIVER_SERIAL=1 runs the sweep points one after another on the calling thread (A/B); so does a
    // profiling session (ace_prof_start): the kernel timer's launch slots are not thread-safe
    const char* ser = getenv("ACE_DRIVER_SERIAL");
    if (n_M == 1 || g_prof.on || (ser && ser[0] == '1')) {
        for (int i = 0; i < n_M; ++i) point(i);
    } else {
        std::vector<std::thread> th;
        th.reserve(n_M);
        for (int i = 0; i < n_M; ++i) th.emplace_back(point, i);
        for (auto& t : th) t.join();
    }
    for (int i = 0; i < n_M; ++i)
        if (rcs[i]) {
            g_err = errs[i];
            return rcs[i];
        }
    return n_M;
}

}  // extern "C"
