/*
 * ace.h -- C-ABI of the MI355X-native 2ACE ADMM channel-recovery hot path.
 *
 * Reference interfaces replaced (reference root: gavinsyw/2ACE-mmWave-Channel-Estimation):
 *
 *  ace_admm_solve_batch   <- [X,Y,converged] = InferADMM(A,B,X0,scale_by_row,use_rank_one,
 *                            tx,rx,lambda,mu0,rho,tol_rel,tol_abs,maxiter,U,D)
 *                            main/src/my_recovery_algorithms/ADMM_v2/inferLowRankV4_multi.m:281
 *                            (A2only Z-prox :423-485) and inferLowRank_Nuclear.m:269
 *                            (nuclear Z-prox :411-439).  One call solves a batch of
 *                            independent realisations; the refinement stage called at
 *                            inferLowRankV4_multi.m:92 / :100 is r = 1, scale_by_row = 1.
 *  ace_admm_solve_host    <- the same, on host arrays (drop-in for MATLAB Engine calls
 *                            that pass matlab.double buffers; main/main.py:427-437).
 *  ace_pipeline_solve_batch <- [X,Y,quality] = inferLowRankV4_multi(A,B,tx,rx)
 *                            main/src/my_recovery_algorithms/ADMM_v2/inferLowRankV4_multi.m:5-109
 *                            (3 restarts), Numerical_Simulation/.../inferLowRankV4.m (1 restart)
 *                            and inferLowRank_Nuclear.m (1 restart, nuclear Z-prox), as called by
 *                            ADMM_v2(meas,FW,TX,RX,version) (ADMM_v2.m:30-32) and
 *                            ADMM_v2_nuclear.m:30-32.  Spectral initialisation (:561-574),
 *                            inferLowRankImpl (:111-271: r = 20 row-scaled stage, rotation by
 *                            eig(X'X), per-column stage), test quality and rank-one retry
 *                            (:68-77), best of restarts (:79-83), refinement (:89-101),
 *                            rollback and rescale (:93-107) -- all on the GPU.
 *  ace_phaselift_solve_batch <- recoveredSig = MyPhaseLift(measurements, measurementMat)
 *                            main/src/my_recovery_algorithms/MyPhaseLift.m:69-107 (TFOCS
 *                            solver_TraceLS + tfocs_AT, prox_trace), batched over realisations.
 *  ace_recover_driver     <- [H_amp,H_angle] = channel_recovery_ADMM_v2_simulation_A2only /
 *                            _A2nuclear / _multiresolution(tx,rx,cb_amp,cb_angle,rss_final,
 *                            seed_id)  main/channel_recovery_ADMM_v2_simulation_A2only.m:9,
 *                            called from main/main.py:427-437 through the MATLAB Engine.
 *  ace_synth_*            <- synthetic trace generation with the semantics of
 *                            main/src/generate_channel/Generate_Channel.m:64-164,
 *                            generate_sensing_matrix/Generate_Sensing_Matrix.m:85-122
 *                            ('Random_Phase_State') and
 *                            generate_measurement/Generate_Measurement.m:67-136.
 *
 * Conventions
 *  - Complex values are complex128, interleaved (re, im) doubles.
 *  - A is row-major [a_shared ? 1 : batch][m][n]; n = tx*rx with the
 *    column-major vec(H) ordering of the reference (element k = i + tx*j).
 *  - Per-realisation vectors are realisation-major: B[batch][m] (f64),
 *    X0/X[batch][n] (c128), Y[batch][m] (c128).
 *  - All pointers passed to ace_admm_solve_batch / ace_synth_* are DEVICE
 *    pointers; the caller owns every buffer (no allocation crosses the ABI).
 *    The workspace must be ace_admm_workspace_size() bytes, 256-B aligned.
 *  - `stream` is a hipStream_t (NULL = default stream).  Calls are
 *    asynchronous on that stream except where noted; they are re-entrant per
 *    stream (no global mutable state besides the thread-local error text).
 *  - Return value 0 = success, negative = error; ace_last_error() returns a
 *    thread-local description of the last error on this thread.
 */
#ifndef ACE_H_
#define ACE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACE_OK 0
#define ACE_ERR_ARG -1        /* invalid argument / shape */
#define ACE_ERR_UNSUPPORTED -2 /* configuration outside the implemented scope */
#define ACE_ERR_HIP -3        /* HIP runtime error */
#define ACE_ERR_WORKSPACE -4  /* workspace too small */

#define ACE_VARIANT_A2ONLY 0  /* inferLowRankV4_multi.m ArgMinZ (rank-profile tail rescale) */
#define ACE_VARIANT_NUCLEAR 1 /* inferLowRank_Nuclear.m ArgMinZ (singular-value soft threshold) */

/* status bits per realisation */
#define ACE_ST_CONVERGED 1u   /* convergence test (inferLowRankV4_multi.m:372) passed */
#define ACE_ST_NO_OPT 2u      /* objective never finite: returned last iterate (reference would raise) */
#define ACE_ST_EIG_NOCONV 4u  /* Z-prox Jacobi hit its sweep cap at least once */
#define ACE_ST_ROLLBACK 8u    /* pipeline: refinement rolled back to X_max (inferLowRankV4_multi.m:94-98) */
#define ACE_ST_RANK_ONE 128u  /* pipeline: the last restart ran the rank-one retry (:73-77), so the refinement
                                 (:92/:100) uses the [1]/[0.95] profile -- set with stop_before_refine too, so a
                                 caller can hand the refinement's flags to ace_admm_cfg::rank_one */

typedef struct ace_admm_cfg {
    int variant;       /* ACE_VARIANT_* */
    int scale_by_row;  /* 1: row-wise magnitude step (:300-308, :344-351); 0: per-column (:352-361).  The two
                          coincide at r = 1 */
    int use_rank_one;  /* ArgMinZ rank profile [1] / [0.95] (inferLowRankV4_multi.m:448-450) for every
                          realisation, unless rank_one is given */
    int maxiter;       /* 500 in the reference (:13) */
    int fixed_iters;   /* 1: throughput mode -- run exactly maxiter iterations (no early exit) */
    int a_shared;      /* 1: one A for the whole batch (shared codebook); 0: private A per realisation */
    int eig_warm;      /* 1: warm-start the Z-prox Jacobi from the previous iteration's eigenvectors */
    int f64_applies;   /* 0: a shared phase-code A (every component in {0, +-c}) runs A v, A^H g and K Y
                          as exact int8 digit-plane products (f64 accuracy); 1: f64 matrix cores always */
    double mu0;        /* 1e-3   (:7) */
    double rho;        /* 1.03   (:8) */
    double tol_rel;    /* 1e-4   (:10) */
    double tol_abs;    /* 1e-8   (:11) */
    int r;             /* columns of X0: 1 (0 = 1) is the refinement stage (:92/:100); up to 32 on a shared A
                          (a_shared = 1): the r-column stages of inferLowRankImpl (:258 row-scaled, :270
                          per-column) */
    int reserved;
    /* Per-realisation use_rank_one [batch] (0/1 bytes, in the same memory space as the solve's other
     * buffers: device for ace_admm_solve_batch, host for ace_admm_solve_host), or NULL: use_rank_one for
     * every realisation.  The refinement of a batch of inferLowRankV4_multi calls passes each call's own
     * last-restart flag (:73-77, :92/:100): ACE_ST_RANK_ONE of ace_pipeline_solve_batch. */
    const uint8_t* rank_one;
} ace_admm_cfg;

/* Fill cfg with the reference defaults (inferLowRankV4_multi.m:6-14), variant A2only,
 * refinement stage (r = 1, scale_by_row = 1), shared A, convergence enabled. */
void ace_admm_cfg_default(ace_admm_cfg* cfg);

/* Workspace bytes needed by ace_admm_solve_batch for this problem (cfg->r columns). */
size_t ace_admm_workspace_size(const ace_admm_cfg* cfg, int batch, int m, int n);

/* Batched InferADMM on device buffers (r = cfg->r columns; R = scale_by_row ? r : 1 output columns).
 *   A      [a_shared?1:batch][m][n] c128      sensing matrix (codebook rows)
 *   B      [batch][m] f64                     RSS magnitudes
 *   X0     [batch][r][n] c128                 initial iterate (column j of realisation b contiguous)
 *   X, Y   [batch][R][n] / [batch][R][m] c128 out  best-objective iterate (opt_X, opt_Y; per-column mode
 *                                             returns the best column, :352-361)
 *   iters  [batch] int32 out (may be NULL)    iterations run
 *   status [batch] uint32 out (may be NULL)   ACE_ST_* bits
 *   mu     [batch] f64 out (may be NULL)      final penalty mu
 * Constraints: n == tx*rx, tx <= 32, rx <= 32 (tx, rx in {4,8,16,32} in the reference; A2only
 * with an odd tx <= 31 is solved as the zero-padded (tx + 1) x rx problem in buffers of its own,
 * `workspace` unused, and returns synchronously), m >= 1, 1 <= r <= 32 (r > 1: shared A only).
 * Returns once all kernels are enqueued; in convergence mode (fixed_iters == 0) the host polls a
 * device flag every few iterations and so synchronises `stream` periodically. */
int ace_admm_solve_batch(const ace_admm_cfg* cfg, int batch, int m, int n, int tx, int rx,
                         const double* A, const double* B, const double* X0,
                         double* X, double* Y, int32_t* iters, uint32_t* status, double* mu,
                         void* workspace, size_t workspace_bytes, void* stream);

/* Host-pointer convenience wrapper: allocates device memory, copies in, solves,
 * copies out, frees.  Synchronous. */
int ace_admm_solve_host(const ace_admm_cfg* cfg, int batch, int m, int n, int tx, int rx,
                        const double* A, const double* B, const double* X0,
                        double* X, double* Y, int32_t* iters, uint32_t* status, double* mu);

/* ---- full recovery pipeline (inferLowRankV4_multi / inferLowRankV4 / inferLowRank_Nuclear) ----
 * MATLAB's randsample (:48), drawn inside every call, is replaced by train partitions: train_idx is a
 * HOST array of 0-based row indices, m_t = floor(m * cc_frac) per restart, in one of two layouts
 * (ace_pipeline_cfg::train_layout):
 *   ACE_TRAIN_SHARED          [restarts][m_t], one partition per restart for the whole batch;
 *   ACE_TRAIN_PER_REALISATION [batch][restarts][m_t], each realisation its own (a Monte-Carlo batch
 *                             of calls, each drawing its own randsample).
 * train_idx = NULL draws per-realisation partitions with the build's counter RNG from
 * ace_pipeline_cfg::train_seed (randperm prefixes, stream b * restarts + restart); it needs
 * train_layout = ACE_TRAIN_PER_REALISATION (ACE_ERR_ARG otherwise: the workspace size follows the layout).  Test rows are the
 * sorted complement (setdiff, :49).  Per-realisation partitions keep the stage state in m-space on the
 * full A (test rows held at zero) and apply (I + K_t)^{-1} through the full (I + K)^{-1} and a
 * per-realisation m_te x m_te block (the Schur identity; m - m_t <= 96, ACE_ERR_UNSUPPORTED beyond: the
 * Python mirror then solves the groups of realisations that share their partitions one call each);
 * realisations whose partitions coincide for every restart take the shared-A_t path.
 * Per realisation, stage_iters holds 4*restarts + 1 counts: for each restart the two
 * inferLowRankImpl stages (:258, :270), then the two stages of the rank-one retry (:73-77;
 * 0 when not run), then the refinement (:92/:100) -- the order of the oracle's stage_iters. */
typedef struct ace_pipeline_cfg {
    int variant;       /* ACE_VARIANT_A2ONLY (keep best restart) or ACE_VARIANT_NUCLEAR (last restart) */
    int restarts;      /* 3 (inferLowRankV4_multi.m:42), 1 (inferLowRankV4, inferLowRank_Nuclear) */
    int r;             /* 20 (:7); clipped to min(r, m, n) (:19), must be <= 32 */
    int maxiter;       /* 500 (:13), every stage */
    int eig_warm;      /* warm-start the Z-prox eigensolver inside each stage */
    int stop_before_refine; /* 0 (reference); 1: return X_max, the refinement's input (:90-92), rescaled
                          (:106-107), with Y_max on the train rows and no refinement stage (its
                          stage_iters column is 0) -- for measuring the unit on the reference's input */
    int train_layout;  /* ACE_TRAIN_SHARED (default) or ACE_TRAIN_PER_REALISATION (see above) */
    int train_seed;    /* seed of the build's draws when train_idx is NULL */
    double mu0;        /* 1e-3 */
    double rho;        /* 1.03 */
    double cc_frac;    /* 0.95 (:10) */
    double tol_rel;    /* 1e-4 */
    double tol_abs;    /* 1e-8 */
} ace_pipeline_cfg;

#define ACE_TRAIN_SHARED 0
#define ACE_TRAIN_PER_REALISATION 1
/* Reference defaults for `variant`: A2only -> 3 restarts, nuclear -> 1 restart. */
void ace_pipeline_cfg_default(ace_pipeline_cfg* cfg, int variant);
/* Workspace bytes for ace_pipeline_solve_batch (0 on invalid arguments).  Not monotonic in batch: a batch
 * of at most 16 realisations runs its restarts concurrently on one workspace copy each, so it can need
 * more than a batch of 17 -- size the workspace for the batch actually passed. */
size_t ace_pipeline_workspace_size(const ace_pipeline_cfg* cfg, int batch, int m, int n);
/* Batched pipeline on device buffers (shared codebook A [m][n] c128, B [batch][m] f64).
 * Outputs: X [batch][n], Y [batch][m] (c128; Y's last m - m_t entries are 0 after a
 * rollback, whose Y_max lives on the train rows), quality [batch] (the LAST restart's, as
 * the reference returns), stage_iters [batch][4*restarts+1], status [batch] (ACE_ST_*).
 * quality, stage_iters and status may be NULL.  Synchronises `stream` once per restart
 * (the rank-one retry set is decided on the host). */
int ace_pipeline_solve_batch(const ace_pipeline_cfg* cfg, int batch, int m, int n, int tx, int rx,
                             const double* A, const double* B, const int32_t* train_idx_host,
                             double* X, double* Y, double* quality, int32_t* stage_iters, uint32_t* status,
                             void* workspace, size_t workspace_bytes, void* stream);
/* The same on host arrays (allocates, copies, solves, frees; synchronous). */
int ace_pipeline_solve_host(const ace_pipeline_cfg* cfg, int batch, int m, int n, int tx, int rx,
                            const double* A, const double* B, const int32_t* train_idx,
                            double* X, double* Y, double* quality, int32_t* stage_iters, uint32_t* status);

/* ---- SpectralInitialize (inferLowRankV4_multi.m:561-574) ----------------------------------
 *   X = SpectralInitialize(A, B, r)
 * for a batch of magnitude vectors B [batch][m] (f64) sharing one A [m][n] (c128, row-major,
 * HOST arrays): X [batch][r][n] c128, column k = sqrt(s_k) v_k for the k-th largest eigenpair of
 * As^H As (As = rows of A scaled by B_i/||a_i||); eigenvectors are defined up to a unit phase
 * (MATLAB's eig and LAPACK pick one; the GPU picks another).  The pipeline's own initialisation
 * (ace_pipeline_solve_batch, :58) runs the same kernels: through the m x m dual Gram when m <= n,
 * the n x n primal Gram otherwise.  status [batch] (may be NULL): ACE_ST_EIG_NOCONV bits.
 * Synchronous; allocates its own device memory. */
int ace_spectral_init_host(int batch, int m, int n, int r, const double* A, const double* B, double* X,
                           uint32_t* status);

/* ---- PhaseLift (MyPhaseLift.m:69-107 via TFOCS solver_TraceLS / tfocs_AT) ----------------
 *   recoveredSig = MyPhaseLift(measurements, measurementMat)
 *   main/src/my_recovery_algorithms/MyPhaseLift.m:69 (called by Recover_Channel.m:34 with
 *   measurements = (rss/2e5).^2*1e10).  A batch of measurement vectors b [batch][m] sharing one
 *   measurement matrix Phi [m][n] (c128, row-major, DEVICE pointers); sig [batch][n] c128 out.
 *   The iteration runs in the coordinates of range(Phi^H) (exact for MyPhaseLift's zero start);
 *   m <= n needs full row rank (else ACE_ERR_UNSUPPORTED).  status: ACE_ST_CONVERGED when the
 *   TFOCS step tolerance stopped the run before maxIts. */
typedef struct ace_phaselift_cfg {
    int maxIts;        /* 4000 (MyPhaseLift.m:82) */
    int restart;       /* 200  (:84) */
    int cntr_reset;    /* 50   (tfocs_initialize.m; 10 when tol < 1e-12) */
    int reserved;
    double tol;        /* 1e-10 (:83), stopCrit 1 */
    double lambda;     /* 5e-2  (:91) */
    double L0, alpha, beta;  /* 1, 0.9, 0.5 (tfocs_initialize.m defaults) */
} ace_phaselift_cfg;
void ace_phaselift_cfg_default(ace_phaselift_cfg* cfg);
size_t ace_phaselift_workspace_size(const ace_phaselift_cfg* cfg, int batch, int m, int n);
int ace_phaselift_solve_batch(const ace_phaselift_cfg* cfg, int batch, int m, int n, const double* Phi,
                              const double* b, double* sig, int32_t* iters, uint32_t* status,
                              void* workspace, size_t workspace_bytes, void* stream);
int ace_phaselift_solve_host(const ace_phaselift_cfg* cfg, int batch, int m, int n, const double* Phi,
                             const double* b, double* sig, int32_t* iters, uint32_t* status);
/* ace_phaselift_solve_host plus solver_TraceLS's result itself (MyPhaseLift.m:98 recoveredMat, the final
 * tfocs_AT iterate): Xr [batch][d][d] c128 (HOST), d = min(m, n), in the coordinates of range(Phi^H)
 * (recoveredMat = Q Xr Q^H, Phi^H = Q R with R = chol(Phi Phi^H); Q = I when m > n).  For parity tests of the
 * iterate and of the TFOCS objective 0.5 ||A(X) - b||^2 + lambda tr X. */
int ace_phaselift_solve_host_x(const ace_phaselift_cfg* cfg, int batch, int m, int n, const double* Phi,
                               const double* b, double* sig, int32_t* iters, uint32_t* status, double* Xr);
/* The prox's eigensolver alone (prox_trace.m:88-92: all eigenpairs of a Hermitian d x d matrix above tau),
 * for parity tests of its paths: A [batch][d][d] c128 (HOST, Hermitian; the lower triangle is read), tau [batch];
 * lam [batch][d] (descending; entries >= k[b] undefined), V [batch][d][d] c128 (eigenvector q as row q),
 * k [batch].  path: 0 unblocked one-stage, 1 blocked one-stage, 2 two-stage (where it applies, else 1); + 4: the
 * vectors of the smaller side of tau (PhaseLift's ACE_PROX_SIDE=1): when more than half of the eigenvalues exceed
 * tau, V holds those at or below it (ascending) and k[b] = -(their count).
 * Synchronous; allocates its own device memory. */
int ace_prox_eig_host(int batch, int d, int path, const double* A, const double* tau, double* lam, double* V,
                      int32_t* k);

/* ---- driver-level boundary (MATLAB Engine calls of main/main.py:308, :427-437) ------------
 *   [H_amp,H_angle] = channel_recovery_ADMM_v2_simulation_<A2only|A2nuclear|multiresolution|phaselift>(
 *                         tx_ant_num, rx_ant_num, cb_amp, cb_angle, rss_final, seed_id)
 *   main/channel_recovery_ADMM_v2_simulation_A2only.m:9-179 (A2nuclear, multiresolution, phaselift
 *   alike; phaselift runs MyPhaseLift per sweep point, Recover_Channel.m:32-35).
 * cb_amp / cb_angle: HOST [P][n] row-major f64 (codebook row p = beam p; MATLAB callers pass
 * the transpose of their P x n arrays), rss_dbm: [P] (dBm).  M_list = NULL selects the
 * reference sweep round(linspace(2, sqrt(4*tx*rx), 8)).^2 (:106-118).  Outputs H_amp, H_angle:
 * HOST [n_M][n] row-major (MATLAB's n_M x 1 x n squeezed), element k in vec(H) order
 * (i + tx*j).  Returns the number of sweep points (>= 1) or a negative error code.
 * Row selection uses the build's RNG seeded from the reference seed lists (MATLAB streams are
 * not reproducible outside MATLAB).  Sweep points with floor(0.95 M) < min(20, M) train rows
 * (M = 4) are ill-posed for the spectral initialisation and return 0 (the reference's
 * NaN -> 0 of :176). */
#define ACE_DRIVER_A2ONLY 0     /* channel_recovery_ADMM_v2_simulation_A2only.m */
#define ACE_DRIVER_A2NUCLEAR 1  /* channel_recovery_ADMM_v2_simulation_A2nuclear.m */
#define ACE_DRIVER_MULTIRES 2   /* channel_recovery_ADMM_v2_simulation_multiresolution.m.  The reference defines the
                                   tiers for 16 x 16 only (rows [1984, 3968, 3968], M <= 96 / <= 256 / else,
                                   ..._multiresolution.m:110-112,137-144); at 32 x 32 the build uses its own analogue
                                   (4x the rows: 7936/15872/15872, thresholds 384/1024) -- a builder-defined layout
                                   whose parity with any reference codebook is unpinned */
#define ACE_DRIVER_PHASELIFT 3  /* channel_recovery_ADMM_v2_simulation_phaselift.m (MyPhaseLift, rng(4096)) */
int ace_recover_driver(int driver, int tx, int rx, int P, const double* cb_amp, const double* cb_angle,
                       const double* rss_dbm, int seed_id, int n_M, const int32_t* M_list,
                       double* H_amp, double* H_angle);
/* The same with the iteration cap of every solve in the call: maxiter > 0 replaces the reference's 500 ADMM
 * iterations per pipeline stage (inferLowRankV4_multi.m:13) or 4000 TFOCS iterations (MyPhaseLift.m:82);
 * 0 keeps them.  For parity runs on the horizon where the reference algorithm is stable against its own
 * rounding (the A2nuclear refinement). */
int ace_recover_driver_ex(int driver, int tx, int rx, int P, const double* cb_amp, const double* cb_angle,
                          const double* rss_dbm, int seed_id, int n_M, const int32_t* M_list, int maxiter,
                          double* H_amp, double* H_angle);
/* The reference M sweep for (tx, rx) into M_out[8]; returns 8 or a negative error code
 * (..._A2only.m:106-118, error :117). */
int ace_driver_m_sweep(int tx, int rx, int32_t* M_out);
/* First k entries of a uniform random permutation of 0..P-1 (randperm(P,k) / randsample,
 * 0-based, sampled order) from the build's counter RNG (seed, stream).  Host only. */
int ace_driver_randperm(uint64_t seed, uint64_t stream, int P, int k, int32_t* out);

/* ---- downstream beamformer ----------------------------------------
 *   wr_out, wt_out = svd_beamformer(H)                       main/codebook_library.py:57-96
 *   wr_out, wt_out = svd_beamformer_compensation(H, offset)  main/codebook_library.py:98-138
 *   reached from codebook_generator (:192-213), H = reshape(H_est[i,:], [tx, rx]) (:197).
 * H: [batch][tx][rx] c128 row-major (DEVICE for _batch), 1 <= tx, rx <= 32 (main.py:454 calls
 * it square; any shape np.shape(H) gives is taken, with zgesdd's QR / LQ / direct paths).
 * offset: [batch][max(tx, rx)] radians (compensation * pi/2; entry k compensates element k of
 * both codes, i.e. numpy's broadcasting — tx != rx admits only a constant row there) or NULL
 * for svd_beamformer.  Outputs: wr_code [batch][rx] and wt_code [batch][tx] (2-bit phase codes
 * 0..3 = the characters of the reference's strings), beam_idx [batch][2] = (tx_idx, rx_idx) of
 * the argmax pair, rss [batch] = its 10*log10(|wt^T H wr|^2 * 1000), status [batch]
 * (ACE_ST_BF_*).  vh_r [batch][rx][rx] / vh_t [batch][tx][tx] (optional, may be NULL): c128 Vh
 * of svd(H) and svd(H^T) in numpy's (zgesdd's) phase and sign convention. */
#define ACE_ST_BF_NONFINITE 16u /* H has NaN/Inf: numpy raises LinAlgError; codes zeroed, beam_idx -1 */
#define ACE_ST_BF_NOCONV 32u    /* dbdsqr iteration budget exhausted (numpy would raise) */
#define ACE_ST_BF_DC 64u        /* min(tx, rx) > 25: zgesdd's divide and conquer, its merge's signs applied;
                                   a vector the merge deflates (rank-deficient H) may still differ */
int ace_svd_beamformer_batch(int batch, int tx, int rx, const double* H, const double* offset,
                             uint8_t* wr_code, uint8_t* wt_code, int32_t* beam_idx, double* rss,
                             uint32_t* status, double* vh_r, double* vh_t, void* stream);
int ace_svd_beamformer_host(int batch, int tx, int rx, const double* H, const double* offset,
                            uint8_t* wr_code, uint8_t* wt_code, int32_t* beam_idx, double* rss,
                            uint32_t* status, double* vh_r, double* vh_t);

/* ---- nuclear-norm prox (A2nuclear ArgMinZ / Shrink) ---------------------------------------
 *   Z = U * Shrink(S, tau) * V'  with [U,S,V] = svd(E)     inferLowRank_Nuclear.m:411-439
 * for a batch of n x r matrices E_b (DEVICE, c128, [batch][r][n]: column j of E_b at
 * E + 2*(b*r + j)*n doubles), r <= 32, tau > 0: the r-general Z-prox kernel of the A2nuclear
 * stages (singular values through the r x r Gram matrix and the Jacobi eigensolver).  Exposed for
 * the prox's own known-answer test; asynchronous on `stream`. */
int ace_nuclear_prox_batch(int batch, int n, int r, const double* E, double tau, double* Z, void* stream);

/* Synthetic traces (device).  Counter-based RNG (splitmix64 of seed/stream/counter),
 * identical integer streams to ace_amd.synth on the host.
 *   ace_synth_codebook: A[count][m][n] c128 with entries exp(j*pi/2*k)/sqrt(n),
 *     k ~ U{0..3}; realisation index base `first` (private A) -- for a shared codebook
 *     pass count = 1, first = -1.
 *   ace_synth_channels: for realisations first..first+count-1: vecH [count][n] c128
 *     (L paths, AoD/AoA ~ U(-47.5deg, 47.5deg), CN gains normalised), B = |A vecH + w|
 *     with w ~ CN(0, 10^(-snr_db/10)), and X0 = vecH + x0_noise * ||vecH||/sqrt(n) * CN(0,1).
 *     A is [a_shared?1:count][m][n]. */
int ace_synth_codebook(uint64_t seed, int64_t first, int count, int m, int n, double* A, void* stream);
int ace_synth_channels(uint64_t seed, int64_t first, int count, int m, int tx, int rx, int L,
                       double snr_db, double x0_noise, const double* A, int a_shared,
                       double* vecH, double* B, double* X0, void* stream);

/* ---- kernel timing (measurement only; no reference counterpart) ----------------
 * Between ace_prof_start and ace_prof_stop every kernel ace_admm_solve_batch
 * enqueues is bracketed by a pair of hipEvents recorded on the launch stream.
 * ace_prof_stop waits for the events and returns, per kernel class, the summed
 * device time (ms) and the number of launches.  Process-global; not thread-safe. */
#define ACE_K_SETUP 0    /* K = A A^H, (I+K)^{-1}, A^H */
#define ACE_K_INIT 1     /* A X0, init, initial Z-prox, K Y */
#define ACE_K_PRE 2      /* V = Z - N/mu, S = Y - M/mu */
#define ACE_K_APPLY_A 3  /* T = S - A V */
#define ACE_K_APPLY_G 4  /* g = G T */
#define ACE_K_YSTEP 5    /* ArgMinY, M update, reductions */
#define ACE_K_APPLY_K 6  /* K Y */
#define ACE_K_APPLY_AH 7 /* X = V + A^H g */
#define ACE_K_ZSTEP 8    /* ArgMinZ, N update, residuals, stop test */
#define ACE_K_FINAL 9
#define ACE_K_MSR 10     /* m-space run: several steady iterations of the unit in one launch */
#define ACE_NKCLASS 11
int ace_prof_start(int max_launches);
/* From the next ace_prof_start on, record only every stride-th launch of each kernel class
 * (default 1) except the classes whose bit (1 << ACE_K_*) is set in full_mask, which are
 * recorded on every launch: keeps the event overhead out of a throughput measurement. */
int ace_prof_sample(int stride, uint32_t full_mask);
int ace_prof_stop(double* total_ms, int32_t* launches);
/* Realisation-iterations the unit solves between the last ace_prof_start / ace_prof_stop pair
 * settled in m-space form (RealState::msp: no apply_AH pass, no Z traffic), for the bench's
 * per-launch work accounting. */
int ace_prof_msp_steps(long long* steps);
/* Algorithmic flops (8 per complex multiply-add) of the launches the last ace_prof_start /
 * ace_prof_stop pair recorded, per kernel class: the GEMM-shaped applies and prox steps of the
 * f64 path (pipeline stages, PhaseLift) carry their count; classes the caller accounts for
 * itself (the unit path's fused kernels) report 0.  flops: [ACE_NKCLASS]. */
int ace_prof_work(double* flops);
/* The same per kernel class, with the launches' algorithmic HBM bytes (every array the step needs read
 * or written once) and int8 matrix-core ops beside the flops; any pointer may be NULL.  Every class
 * of the pipeline's r-column stages (the int8 digit-plane applies, the r-column Z-step, the Y-step,
 * the pre-pass) carries its bytes, so the dominant class by device time has a roofline. */
int ace_prof_work_ex(double* flops, double* bytes, double* int8_ops);

/* InferADMM solves (unit solves and every pipeline stage) per apply path since the last reset,
 * process-wide: counts[0] shared phase-code codebook on the exact int8 digit-plane applies,
 * counts[1] private phase-code codebooks (2-bit code images), counts[2] f64 applies on a shared
 * A, counts[3] f64 applies on private A.  reset != 0 zeroes the counters after reading them;
 * counts may be NULL.  Tells a caller whether its codebook reached the phase-code path. */
int ace_path_counts(int64_t* counts, int reset);

/* Dynamic LDS (bytes) the launcher of `kernel` requests at operand size `m` (host arithmetic, no
 * GPU call): "i8ah" (apply_AH), "i8ah_fuse", "i8ah_ky" (K Y), "gyk", "gyf", "msr", "nms" (m = the
 * measurement count), "hetrd", "hetrd_blk" (m = the Hermitian order).  With the kernel's static LDS
 * (compiler resource report) it must stay within the CU's 160 KiB for every shape the path takes;
 * tests/test_lds_budget.py checks that.  ACE_ERR_ARG for an unknown name. */
int ace_lds_request(const char* kernel, int m, size_t* bytes);

/* Last error text for this thread ("" if none). */
const char* ace_last_error(void);

/* Library version string. */
const char* ace_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ACE_H_ */
