// Batched recovery pipeline: inferLowRankV4_multi (main/src/my_recovery_algorithms/
// ADMM_v2/inferLowRankV4_multi.m:5-109), inferLowRankV4 (Numerical_Simulation, one
// restart) and inferLowRank_Nuclear (one restart, nuclear Z-prox), every stage on the GPU.
//
//   :27-38   A_norm = ||A||_F/sqrt(m), B_norm = ||B|| per realisation      anorm/bnorm
//   :42-53   per restart: train rows (caller's partition), test = setdiff   gather_rows/_b
//   :58      SpectralInitialize on (A_t, B_t)                               ace_spectral.hip + GEMM
//   :65      inferLowRankImpl (U = inv(A_t'A_t+I) as Woodbury K_t, G_t;
//            r-column row-scaled ADMM :258, X = X eig(X'X) :263-264,
//            per-column ADMM :270, best column)                             admm_run x2, gram_rotate
//   :68      quality on the test rows                                      quality
//   :73-77   rank-one retry for realisations with quality < 0.6: the retry
//            set is gathered into a contiguous sub-batch and scattered back  move_rows
//   :79-83   best of restarts (A2only; the nuclear driver keeps the last)   keep_best
//   :89-101  refinement on the full A at r = 1 with the last restart's
//            use_rank_one (per realisation)                                 admm_run (fast r = 1 path)
//   :93-107  rollback when the last quality > 0.6 and the similarity < 0.6; rescale   finish
#include <algorithm>
#include <cstring>

#include <thread>

#include "ace_host.hpp"
#include "ace_pipe.hpp"

using namespace ace;

namespace {

// status bits a stage contributes to the pipeline status (its CONVERGED bit does not)
constexpr unsigned kStageBits = ACE_ST_NO_OPT | ACE_ST_EIG_NOCONV;

struct PipeDims {
    int batch, m, n, tx, rx, r, mt, mte, restarts;
    bool part;     // per-realisation partitions: m-space stage state on the full A (PartRows)
    int ldmask;    // row stride of the train-row masks
};

// The pieces one restart (:42-77) works on.  Restarts are independent until the best of them is
// taken (:79-83), so a small batch (the driver's one realisation per sweep point) runs them
// concurrently, each on its own stream and workspace copy; a large batch, which fills the GPU on
// its own, runs them one after another in one copy.
struct RestartWs {
    double *Bt, *Bte, *Bt_s, *Bte_s, *At, *Ate;
    LinOps Lt;
    double *W, *spec, *Xs, *Xs_s;
    double *X1, *Y1;                 // stage-1 output (r columns), reused by both stages' chains
    double *X2, *Y2, *X2_s, *Y2_s;   // impl outputs (best column); Y2 on the train rows in sampled order
    double *q, *q_s;
    int *iters, *stat, *idx_rows, *idx_sub, *status_dev;
    unsigned char* rank_one;
    AdmmState sr;                    // r-column state (m_t rows; m rows with per-realisation partitions)
    // per-realisation partitions (PipeDims::part): the restart's PartRows tables, their retry-subset
    // copies, the subset's B rows, the spectral W in m-space and the stages' m-space Y outputs
    int *rows, *rows_s;
    unsigned char *mask, *mask_s;
    double *geinv, *geinv_s, *Bn_s, *Wm, *Y2m, *Y2m_s;
};

constexpr int kConcurrentBatch = 16;   // restarts run concurrently up to this batch size
int restart_copies(const PipeDims& d) {
    static const bool serial = [] {
        const char* e = getenv("ACE_PIPE_SERIAL");
        return e && e[0] == '1';
    }();
    return (!serial && d.restarts > 1 && d.batch <= kConcurrentBatch) ? d.restarts : 1;
}

struct PipeWs {
    double *anorm, *bnorm, *Bn, *An;
    LinOps Lf;
    double *qmax, *qlast, *Xmax, *Ymax, *Xr, *Yr;
    int *iters, *stat, *idx_all, *stage_dev, *status_dev;
    unsigned char* rank_one;         // the refinement's use_rank_one (the last restart's)
    AdmmState s1;                    // refinement state (r = 1, m rows)
    int nrw;
    RestartWs rw[16];
};

void restart_carve(Carver& cv, const PipeDims& d, RestartWs* w) {
    const size_t cz = 16, B = (size_t)d.batch;
    const int md = d.part ? d.m : d.mt;   // rows of the stage state
    *w = RestartWs{};
    if (!d.part) {
        w->Bt = cv.take(8 * B * d.mt);
        w->Bte = cv.take(8 * B * std::max(d.mte, 1));
        w->Bt_s = cv.take(8 * B * d.mt);
        w->Bte_s = cv.take(8 * B * std::max(d.mte, 1));
        w->At = cv.take(cz * d.mt * d.n);
        w->Ate = cv.take(cz * std::max(d.mte, 1) * d.n);
        linops_carve(cv, true, d.batch, d.mt, d.n, &w->Lt);
        w->spec = cv.take(spectral_scratch_bytes(d.mt, d.n, d.batch, d.r));
    } else {
        const size_t te2 = (size_t)std::max(d.mte, 1) * std::max(d.mte, 1);
        w->rows = cv.take<int>(4 * B * d.m);
        w->rows_s = cv.take<int>(4 * B * d.m);
        w->mask = cv.take<unsigned char>(B * d.ldmask);
        w->mask_s = cv.take<unsigned char>(B * d.ldmask);
        w->geinv = cv.take(cz * B * te2);
        w->geinv_s = cv.take(cz * B * te2);
        w->Bn_s = cv.take(8 * B * d.m);
        w->Wm = cv.take(cz * B * d.r * d.m);
        w->Y2m = cv.take(cz * B * d.m);
        w->Y2m_s = cv.take(cz * B * d.m);
        // the primal form reads the full A^H and B (m rows): size for both forms
        w->spec = cv.take(std::max(spectral_scratch_bytes(d.mt, d.n, d.batch, d.r),
                                   spectral_scratch_bytes(d.m, d.n, d.batch, d.r)));
    }
    w->W = cv.take(cz * B * d.r * d.mt);
    w->Xs = cv.take(cz * B * d.r * d.n);
    w->Xs_s = cv.take(cz * B * d.r * d.n);
    w->X1 = cv.take(cz * B * d.r * d.n);
    w->Y1 = cv.take(cz * B * d.r * md);
    w->X2 = cv.take(cz * B * d.n);
    w->Y2 = cv.take(cz * B * d.mt);
    w->X2_s = cv.take(cz * B * d.n);
    w->Y2_s = cv.take(cz * B * d.mt);
    w->q = cv.take(8 * B);
    w->q_s = cv.take(8 * B);
    w->iters = cv.take<int>(4 * B);
    w->stat = cv.take<int>(4 * B);
    w->idx_rows = cv.take<int>(4 * (size_t)d.m);
    w->idx_sub = cv.take<int>(4 * B);
    w->status_dev = cv.take<int>(4 * B);
    w->rank_one = cv.take<unsigned char>(B);
    admm_state_carve(cv, d.batch, md, d.n, d.r, &w->sr);
}

void pipe_carve(Carver& cv, const PipeDims& d, PipeWs* w) {
    const size_t cz = 16, B = (size_t)d.batch;
    w->anorm = cv.take(256);
    w->bnorm = cv.take(8 * B);
    w->Bn = cv.take(8 * B * d.m);
    w->An = cv.take(cz * d.m * d.n);
    linops_carve(cv, true, d.batch, d.m, d.n, &w->Lf);
    w->qmax = cv.take(8 * B);
    w->qlast = cv.take(8 * B);
    w->Xmax = cv.take(cz * B * d.n);
    w->Ymax = cv.take(cz * B * d.mt);
    w->Xr = cv.take(cz * B * d.n);
    w->Yr = cv.take(cz * B * d.m);
    w->iters = cv.take<int>(4 * B);
    w->stat = cv.take<int>(4 * B);
    w->idx_all = cv.take<int>(4 * (size_t)d.m);
    w->stage_dev = cv.take<int>(4 * B * (4 * d.restarts + 1));
    w->status_dev = cv.take<int>(4 * B);
    w->rank_one = cv.take<unsigned char>(B);
    admm_state_carve(cv, d.batch, d.m, d.n, 1, &w->s1);
    w->nrw = restart_copies(d);
    for (int i = 0; i < w->nrw; ++i) restart_carve(cv, d, &w->rw[i]);
}

int validate_dims(const ace_pipeline_cfg* c, int batch, int m, int n, PipeDims* d) {
    if (!c) return fail(ACE_ERR_ARG, "cfg is NULL");
    if (batch < 1 || m < 1 || n < 1) return fail(ACE_ERR_ARG, "batch/m/n must be >= 1 (got %d/%d/%d)", batch, m, n);
    if (c->variant != ACE_VARIANT_A2ONLY && c->variant != ACE_VARIANT_NUCLEAR)
        return fail(ACE_ERR_ARG, "unknown variant %d", c->variant);
    if (c->restarts < 1 || c->restarts > 16) return fail(ACE_ERR_ARG, "restarts must be in [1,16]");
    if (c->maxiter < 1) return fail(ACE_ERR_ARG, "maxiter must be >= 1");
    if (!(c->mu0 > 0) || !(c->rho > 0)) return fail(ACE_ERR_ARG, "mu0 and rho must be > 0");
    if (!(c->cc_frac > 0) || !(c->cc_frac <= 1)) return fail(ACE_ERR_ARG, "cc_frac must be in (0, 1]");
    const int r = std::min(std::min(c->r, m), n);                     // :19
    const int mt = (int)std::floor((double)m * c->cc_frac);           // :48
    if (r < 1 || r > 32) return fail(ACE_ERR_UNSUPPORTED, "r = min(r, m, n) must be in [1, 32] (got %d)", r);
    if (mt < r)
        return fail(ACE_ERR_UNSUPPORTED, "floor(m*cc_frac) = %d train rows < r = %d: the spectral initialisation "
                    "would take eigenvectors of the null space (ill-posed, not supported)", mt, r);
    if (std::min(mt, n) > 1600)
        return fail(ACE_ERR_UNSUPPORTED, "min(train rows %d, n %d) > 1600 (spectral tridiagonalisation LDS limit)", mt, n);
    if (n > 4096) return fail(ACE_ERR_UNSUPPORTED, "n must be <= 4096 (got %d)", n);
    *d = PipeDims{batch, m, n, 0, 0, r, mt, m - mt, c->restarts, false, (m + 7) & ~7};
    return ACE_OK;
}

int validate(const ace_pipeline_cfg* c, int batch, int m, int n, int tx, int rx, PipeDims* d) {
    ACE_TRY(validate_dims(c, batch, m, n, d));
    if (tx * rx != n) return fail(ACE_ERR_ARG, "n (%d) != tx*rx (%d*%d)", n, tx, rx);
    if (tx < 2 || tx > 32 || (tx & 1) || rx > 32)
        return fail(ACE_ERR_UNSUPPORTED, "pipeline needs even tx in [2,32] and rx <= 32 (got %d, %d)", tx, rx);
    d->tx = tx;
    d->rx = rx;
    return ACE_OK;
}

// inferLowRankImpl (:111-271) for `nb` realisations: Xs [nb][r][n], Bt [nb][mt] ->
// X2 [nb][n], Y2 [nb][mt] (best column of the per-column stage); iteration counts of the
// two stages into stage_dev columns col, col + 1 (rows idx[k] or k).
int run_impl(const PipeDims& d, RestartWs& w, const LinOps& L, const PartRows* pr, int* stage_dev,
             const AdmmParams& base, int nb, const double* Xs, const double* Bt, double* X2, double* Y2, const int* idx,
             int col, hipStream_t st) {
    const int ld = 4 * d.restarts + 1;
    AdmmParams p = base;
    p.r = d.r;
    p.row_mode = 1;                                               // :258 scale_by_row = true
    p.part = pr;
    ACE_TRY(admm_run(L, p, w.sr, nb, Bt, Xs, w.X1, w.Y1, w.iters, (uint32_t*)w.stat, nullptr, st));
    launch_put_col(nb, w.iters, idx, stage_dev, ld, col, 0, st);
    launch_put_col(nb, w.stat, idx, w.status_dev, 1, 0, kStageBits, st);
    launch_gram_rotate(d.n, d.r, nb, w.X1, nullptr, st);         // :263-264
    p.row_mode = 0;                                               // :270 scale_by_row = false
    ACE_TRY(admm_run(L, p, w.sr, nb, Bt, w.X1, X2, Y2, w.iters, (uint32_t*)w.stat, nullptr, st));
    launch_put_col(nb, w.iters, idx, stage_dev, ld, col + 1, 0, st);
    launch_put_col(nb, w.stat, idx, w.status_dev, 1, 0, kStageBits, st);
    ACE_LAUNCHED("r-column stage");
    return ACE_OK;
}

// One restart (:42-77) for the whole batch on stream st: partition, K_t / G_t, SpectralInitialize,
// inferLowRankImpl, test quality, rank-one retry.  Leaves q, X2, Y2, rank_one and the restart's
// status bits in w.
int run_restart(int i, const PipeDims& d, const double* A, const double* anorm, const double* Bn,
                const std::vector<int>& rows, const AdmmParams& base, RestartWs& w, int* stage_dev, hipStream_t st) {
    const int batch = d.batch, n = d.n, m = d.m;
    ACE_HIP(hipMemsetAsync(w.status_dev, 0, 4 * (size_t)batch, st));
    // ---- :47-53 partition
    ACE_HIP(upload(w.idx_rows, rows.data(), 4 * (size_t)m, st));
    launch_gather_rows(d.mt, n, A, w.idx_rows, anorm, w.At, st);
    launch_gather_rows(d.mte, n, A, w.idx_rows + d.mt, anorm, w.Ate, st);
    launch_gather_b(m, d.mt, batch, Bn, w.idx_rows, w.Bt, st);
    launch_gather_b(m, d.mte, batch, Bn, w.idx_rows + d.mt, w.Bte, st);
    w.Lt.A = w.At;
    ACE_TRY(linops_setup(w.Lt, batch, st));                          // K_t, G_t (U, :242), A_t^H
    // ---- :58 SpectralInitialize: X = V(:, 1:r) diag(sqrt(s))
    {
        ProfScope ps(ACE_K_SETUP, st);
        if (spectral_primal(d.mt, n)) {
            if (launch_spectral_primal(d.mt, n, d.r, batch, w.Lt.K, w.Lt.AH, w.Bt, w.spec, w.Xs, w.status_dev, st))
                return fail(ACE_ERR_UNSUPPORTED, "spectral initialisation: n = %d too large", n);
        } else {
            if (launch_spectral(d.mt, d.r, batch, w.Lt.K, w.Bt, w.spec, w.W, w.status_dev, st))
                return fail(ACE_ERR_UNSUPPORTED, "spectral initialisation: m_t = %d too large", d.mt);
            launch_zgemm(0, false, n, d.mt, batch * d.r, w.Lt.AH, d.mt, 0, w.W, d.mt, 0, w.Xs, nullptr, n, 0, 1, st);
        }
    }
    ACE_LAUNCHED("spectral initialisation");
    // ---- :65-68 impl (use_rank_one = false) and test quality
    AdmmParams p = base;
    p.use_rank_one = 0;
    p.rank_one = nullptr;
    ACE_TRY(run_impl(d, w, w.Lt, nullptr, stage_dev, p, batch, w.Xs, w.Bt, w.X2, w.Y2, nullptr, 4 * i, st));
    launch_quality(n, d.mte, batch, w.Ate, w.X2, w.Bte, w.q, st);
    // ---- :73-77 rank-one retry on the realisations with quality < 0.6
    std::vector<double> hq(batch);
    std::vector<unsigned char> ro(batch);
    std::vector<int> fails;
    ACE_HIP(read_back(hq.data(), w.q, 8 * (size_t)batch, st));
    for (int b = 0; b < batch; ++b) {
        ro[b] = hq[b] < 0.6;
        if (ro[b]) fails.push_back(b);
    }
    ACE_HIP(upload(w.rank_one, ro.data(), batch, st));
    const int nf = (int)fails.size();
    if (nf > 0) {
        ACE_HIP(upload(w.idx_sub, fails.data(), 4 * (size_t)nf, st));
        launch_move_rows(nf, 2LL * d.r * n, w.Xs, w.Xs_s, w.idx_sub, false, st);
        launch_move_rows(nf, d.mt, w.Bt, w.Bt_s, w.idx_sub, false, st);
        launch_move_rows(nf, std::max(d.mte, 1), w.Bte, w.Bte_s, w.idx_sub, false, st);
        p.use_rank_one = 1;
        ACE_TRY(run_impl(d, w, w.Lt, nullptr, stage_dev, p, nf, w.Xs_s, w.Bt_s, w.X2_s, w.Y2_s, w.idx_sub, 4 * i + 2, st));
        launch_quality(n, d.mte, nf, w.Ate, w.X2_s, w.Bte_s, w.q_s, st);
        launch_move_rows(nf, 2LL * n, w.X2_s, w.X2, w.idx_sub, true, st);
        launch_move_rows(nf, 2LL * d.mt, w.Y2_s, w.Y2, w.idx_sub, true, st);
        launch_move_rows(nf, 1, w.q_s, w.q, w.idx_sub, true, st);
    }
    ACE_LAUNCHED("restart selection");
    return ACE_OK;
}

// One restart with per-realisation partitions (PipeDims::part): the same steps on the full normalised A
// (Lf: K, G = (I + K)^{-1}, A^H and its int8 images, built once for the call), each realisation's rows
// in PartRows.  prow [batch][m] (train rows in sampled order, then the test rows ascending) and pmask
// [batch][ldmask] are the host tables of this restart.
int run_restart_part(int i, const PipeDims& d, const LinOps& Lf, const double* An, const double* Bn,
                     const std::vector<int>& prow, const std::vector<unsigned char>& pmask, const AdmmParams& base,
                     RestartWs& w, int* stage_dev, hipStream_t st) {
    const int batch = d.batch, n = d.n, m = d.m;
    ACE_HIP(hipMemsetAsync(w.status_dev, 0, 4 * (size_t)batch, st));
    ACE_HIP(upload(w.rows, prow.data(), 4 * (size_t)batch * m, st));
    ACE_HIP(upload(w.mask, pmask.data(), (size_t)batch * d.ldmask, st));
    const PartRows pr{w.rows, w.mask, w.geinv, m, d.mt, d.ldmask};
    launch_part_geinv(batch, pr, Lf.G, w.geinv, w.status_dev, st);   // (I + K_t)^{-1} via G_ee^{-1}
    // ---- :58 SpectralInitialize on each realisation's train rows
    {
        ProfScope ps(ACE_K_SETUP, st);
        if (spectral_primal(d.mt, n)) {
            if (launch_spectral_primal(d.mt, n, d.r, batch, Lf.K, Lf.AH, Bn, w.spec, w.Xs, w.status_dev, st, &pr))
                return fail(ACE_ERR_UNSUPPORTED, "spectral initialisation: n = %d too large", n);
        } else {
            if (launch_spectral(d.mt, d.r, batch, Lf.K, Bn, w.spec, w.W, w.status_dev, st, &pr))
                return fail(ACE_ERR_UNSUPPORTED, "spectral initialisation: m_t = %d too large", d.mt);
            launch_part_expand(batch, d.r, pr, w.W, w.Wm, st);      // X = A_t^H W = A^H W~
            launch_zgemm(0, false, n, m, batch * d.r, Lf.AH, m, 0, w.Wm, m, 0, w.Xs, nullptr, n, 0, 1, st);
        }
    }
    ACE_LAUNCHED("spectral initialisation (per-realisation partitions)");
    // ---- :65-68 impl (use_rank_one = false) and test quality
    AdmmParams p = base;
    p.use_rank_one = 0;
    p.rank_one = nullptr;
    ACE_TRY(run_impl(d, w, Lf, &pr, stage_dev, p, batch, w.Xs, Bn, w.X2, w.Y2m, nullptr, 4 * i, st));
    launch_part_compact(batch, 1, pr, w.Y2m, w.Y2, st);
    launch_part_quality(n, batch, pr, An, w.X2, Bn, w.q, st);
    // ---- :73-77 rank-one retry on the realisations with quality < 0.6
    std::vector<double> hq(batch);
    std::vector<unsigned char> ro(batch);
    std::vector<int> fails;
    ACE_HIP(read_back(hq.data(), w.q, 8 * (size_t)batch, st));
    for (int b = 0; b < batch; ++b) {
        ro[b] = hq[b] < 0.6;
        if (ro[b]) fails.push_back(b);
    }
    ACE_HIP(upload(w.rank_one, ro.data(), batch, st));
    const int nf = (int)fails.size();
    if (nf > 0) {
        const long long te2 = (long long)std::max(d.mte, 1) * std::max(d.mte, 1);
        ACE_HIP(upload(w.idx_sub, fails.data(), 4 * (size_t)nf, st));
        launch_move_rows(nf, 2LL * d.r * n, w.Xs, w.Xs_s, w.idx_sub, false, st);
        launch_move_rows(nf, m, Bn, w.Bn_s, w.idx_sub, false, st);
        launch_move_rows(nf, 2 * te2, w.geinv, w.geinv_s, w.idx_sub, false, st);
        launch_move_bytes(nf, 4LL * m, w.rows, w.rows_s, w.idx_sub, false, st);
        launch_move_bytes(nf, d.ldmask, w.mask, w.mask_s, w.idx_sub, false, st);
        const PartRows prs{w.rows_s, w.mask_s, w.geinv_s, m, d.mt, d.ldmask};
        p.use_rank_one = 1;
        ACE_TRY(run_impl(d, w, Lf, &prs, stage_dev, p, nf, w.Xs_s, w.Bn_s, w.X2_s, w.Y2m_s, w.idx_sub, 4 * i + 2, st));
        launch_part_compact(nf, 1, prs, w.Y2m_s, w.Y2_s, st);
        launch_part_quality(n, nf, prs, An, w.X2_s, w.Bn_s, w.q_s, st);
        launch_move_rows(nf, 2LL * n, w.X2_s, w.X2, w.idx_sub, true, st);
        launch_move_rows(nf, 2LL * d.mt, w.Y2_s, w.Y2, w.idx_sub, true, st);
        launch_move_rows(nf, 1, w.q_s, w.q, w.idx_sub, true, st);
    }
    ACE_LAUNCHED("restart selection (per-realisation partitions)");
    return ACE_OK;
}

// The restarts' partitions from the caller's train_idx (or the build's RNG) in the layout the solve
// runs: shared [restarts][m_t] rows + test complements, or per-realisation PartRows tables.
struct Partitions {
    bool part = false;
    std::vector<std::vector<int>> rows;               // shared: [restarts] -> train then test rows
    std::vector<std::vector<int>> prow;               // part: [restarts] -> [batch][m]
    std::vector<std::vector<unsigned char>> pmask;    // part: [restarts] -> [batch][ldmask]
};

int check_partition(const int32_t* tr, int m, int mt, std::vector<int>& out, std::vector<char>& seen, int b, int i) {
    std::fill(seen.begin(), seen.end(), 0);
    out.clear();
    for (int k = 0; k < mt; ++k) {
        const int v = tr[k];
        if (v < 0 || v >= m || seen[v])
            return fail(ACE_ERR_ARG, "train_idx[%d][%d][%d] = %d: out of range or repeated", b, i, k, v);
        seen[v] = 1;
        out.push_back(v);
    }
    for (int v = 0; v < m; ++v)
        if (!seen[v]) out.push_back(v);
    return ACE_OK;
}

int build_partitions(const ace_pipeline_cfg* cfg, const PipeDims& d0, const int32_t* train_idx, Partitions* P) {
    const int B = d0.batch, R = d0.restarts, m = d0.m, mt = d0.mt;
    const bool each = train_idx == nullptr || cfg->train_layout == ACE_TRAIN_PER_REALISATION;
    std::vector<int32_t> drawn;
    if (!train_idx) {   // randsample per call (:48) from the build's counter RNG
        drawn.resize((size_t)B * R * mt);
        for (int b = 0; b < B; ++b)
            for (int i = 0; i < R; ++i)
                (void)ace_driver_randperm((uint64_t)(uint32_t)cfg->train_seed, (uint64_t)b * R + i, m, mt,
                                          drawn.data() + ((size_t)b * R + i) * mt);
        train_idx = drawn.data();
    }
    bool same = true;   // per-realisation partitions that coincide everywhere take the shared path
    if (each)
        for (int b = 1; b < B && same; ++b)
            same = std::equal(train_idx, train_idx + (size_t)R * mt, train_idx + (size_t)b * R * mt);
    P->part = each && !same;
    std::vector<char> seen(m);
    std::vector<int> rw;
    if (!P->part) {
        P->rows.assign(R, {});
        for (int i = 0; i < R; ++i) ACE_TRY(check_partition(train_idx + (size_t)i * mt, m, mt, P->rows[i], seen, 0, i));
        return ACE_OK;
    }
    if (m - mt > PART_MAXTE)
        return fail(ACE_ERR_UNSUPPORTED, "per-realisation partitions need m - m_t <= %d test rows (got %d)", PART_MAXTE,
                    m - mt);
    const int ldm = d0.ldmask;
    P->prow.assign(R, std::vector<int>((size_t)B * m));
    P->pmask.assign(R, std::vector<unsigned char>((size_t)B * ldm, 0));
    for (int b = 0; b < B; ++b)
        for (int i = 0; i < R; ++i) {
            ACE_TRY(check_partition(train_idx + ((size_t)b * R + i) * mt, m, mt, rw, seen, b, i));
            std::copy(rw.begin(), rw.end(), P->prow[i].begin() + (size_t)b * m);
            for (int k = 0; k < mt; ++k) P->pmask[i][(size_t)b * ldm + rw[k]] = 1;
        }
    return ACE_OK;
}

}  // namespace

extern "C" {

int ace_spectral_init_host(int batch, int m, int n, int r, const double* A, const double* B, double* X,
                           uint32_t* status) {
    g_err.clear();
    if (!A || !B || !X) return fail(ACE_ERR_ARG, "NULL buffer");
    if (batch < 1 || m < 1 || n < 1 || r < 1) return fail(ACE_ERR_ARG, "batch/m/n/r must be >= 1");
    if (r > 32 || r > m || r > n) return fail(ACE_ERR_UNSUPPORTED, "r must be <= min(32, m, n) (got %d)", r);
    if (std::min(m, n) > 1600) return fail(ACE_ERR_UNSUPPORTED, "min(m, n) = %d > 1600 (LDS limit)", std::min(m, n));
    const bool primal = spectral_primal(m, n);
    const size_t nA = 16 * (size_t)m * n, nK = 16 * (size_t)m * m, nB = 8 * (size_t)batch * m,
                 nW = 16 * (size_t)batch * r * m, nX = 16 * (size_t)batch * r * n,
                 nS = spectral_scratch_bytes(m, n, batch, r);
    std::vector<void*> bufs;
    struct Free {
        std::vector<void*>& b;
        hipStream_t st = nullptr;
        ~Free() {
            if (st) {
                (void)hipStreamSynchronize(st);
                (void)hipStreamDestroy(st);
            }
            for (void* p : b) (void)hipFree(p);
        }
    } guard{bufs};
    auto dalloc = [&](size_t bytes) -> double* {
        void* p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
        bufs.push_back(p);
        return static_cast<double*>(p);
    };
    double *dA = dalloc(nA), *dAH = dalloc(nA), *dK = dalloc(nK), *dB = dalloc(nB), *dW = dalloc(primal ? 16 : nW),
           *dX = dalloc(nX), *dS = dalloc(nS);
    int* dst = reinterpret_cast<int*>(dalloc(4 * (size_t)batch));
    if (!dA || !dAH || !dK || !dB || !dW || !dX || !dS || !dst) return fail(ACE_ERR_HIP, "device allocation failed");
    ACE_HIP(hipStreamCreateWithFlags(&guard.st, hipStreamNonBlocking));
    hipStream_t st = guard.st;
    ACE_HIP(upload(dA, A, nA, st));
    ACE_HIP(upload(dB, B, nB, st));
    ACE_HIP(hipMemsetAsync(dst, 0, 4 * (size_t)batch, st));
    launch_conj_transpose(m, n, dA, dAH, st);
    launch_zgemm(0, true, m, n, m, dA, n, 0, dA, n, 0, dK, nullptr, m, 0, 1, st);   // K = A A^H
    if (primal) {
        if (launch_spectral_primal(m, n, r, batch, dK, dAH, dB, dS, dX, dst, st))
            return fail(ACE_ERR_UNSUPPORTED, "spectral initialisation: n = %d too large", n);
    } else {
        if (launch_spectral(m, r, batch, dK, dB, dS, dW, dst, st))
            return fail(ACE_ERR_UNSUPPORTED, "spectral initialisation: m = %d too large", m);
        launch_zgemm(0, false, n, m, batch * r, dAH, m, 0, dW, m, 0, dX, nullptr, n, 0, 1, st);
    }
    ACE_LAUNCHED("nuclear spectral initialisation");
    ACE_HIP(read_back(X, dX, nX, st));
    if (status) ACE_HIP(read_back(status, dst, 4 * (size_t)batch, st));
    return ACE_OK;
}


void ace_pipeline_cfg_default(ace_pipeline_cfg* c, int variant) {
    std::memset(c, 0, sizeof *c);
    c->variant = variant;
    c->restarts = variant == ACE_VARIANT_NUCLEAR ? 1 : 3;
    c->r = 20;
    c->maxiter = 500;
    c->eig_warm = 1;
    c->mu0 = 1e-3;
    c->rho = 1.03;
    c->cc_frac = 0.95;
    c->tol_rel = 1e-4;
    c->tol_abs = 1e-8;
}

size_t ace_pipeline_workspace_size(const ace_pipeline_cfg* cfg, int batch, int m, int n) {
    PipeDims d;
    const std::string keep = g_err;
    if (validate_dims(cfg, batch, m, n, &d)) {
        g_err = keep;
        return 0;
    }
    Carver cv{nullptr};
    PipeWs w;
    pipe_carve(cv, d, &w);
    size_t need = cv.off + 256;
    if (cfg->train_layout == ACE_TRAIN_PER_REALISATION) {   // either form, as the partitions decide
        Carver cp{nullptr};
        d.part = true;
        pipe_carve(cp, d, &w);
        need = std::max(need, cp.off + 256);
    }
    return need;
}

int ace_pipeline_solve_batch(const ace_pipeline_cfg* cfg, int batch, int m, int n, int tx, int rx, const double* A,
                             const double* B, const int32_t* train_idx, double* Xo, double* Yo, double* quality,
                             int32_t* stage_iters, uint32_t* status, void* workspace, size_t workspace_bytes,
                             void* stream) {
    g_err.clear();
    PipeDims d;
    ACE_TRY(validate(cfg, batch, m, n, tx, rx, &d));
    if (!A || !B || !Xo || !Yo || !workspace) return fail(ACE_ERR_ARG, "NULL buffer");
    if (cfg->train_layout != ACE_TRAIN_SHARED && cfg->train_layout != ACE_TRAIN_PER_REALISATION)
        return fail(ACE_ERR_ARG, "unknown train_layout %d", cfg->train_layout);
    // the build's draws are per realisation: ace_pipeline_workspace_size sizes that form only for that layout
    if (!train_idx && cfg->train_layout != ACE_TRAIN_PER_REALISATION)
        return fail(ACE_ERR_ARG, "train_idx = NULL (the build's per-realisation draws) needs train_layout = "
                                 "ACE_TRAIN_PER_REALISATION");
    // partitions (host): train rows in sampled order, test rows = sorted complement (:48-49)
    Partitions P;
    ACE_TRY(build_partitions(cfg, d, train_idx, &P));
    d.part = P.part;
    hipStream_t st = (hipStream_t)stream;
    Carver sz{nullptr};
    PipeWs w;
    pipe_carve(sz, d, &w);
    if (sz.off + 256 > workspace_bytes)
        return fail(ACE_ERR_WORKSPACE, "workspace too small: need %zu bytes, got %zu", sz.off + 256, workspace_bytes);
    poison_workspace(workspace, workspace_bytes, st);
    Carver cv{(char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255)};
    pipe_carve(cv, d, &w);
    const int ld = 4 * d.restarts + 1;

    AdmmParams base{};
    base.variant = cfg->variant;
    base.maxiter = cfg->maxiter;
    base.fixed_iters = 0;
    base.eig_warm = cfg->eig_warm;
    base.mu0 = cfg->mu0;
    base.rho = cfg->rho;
    base.tol_rel = cfg->tol_rel;
    base.tol_abs = cfg->tol_abs;
    base.tx = tx;
    base.rx = rx;

    // ---- :27-38 normalisation
    std::vector<int> iota(m);
    for (int i = 0; i < m; ++i) iota[i] = i;
    launch_anorm(m, n, A, cfg->tol_abs, w.anorm, st);
    ACE_HIP(upload(w.idx_all, iota.data(), 4 * (size_t)m, st));
    launch_gather_rows(m, n, A, w.idx_all, w.anorm, w.An, st);
    launch_bnorm(m, batch, B, cfg->tol_abs, w.bnorm, w.Bn, st);
    launch_fill(batch, -1.0, w.qmax, st);                                 // max_quality = -1 (:40)
    ACE_HIP(hipMemsetAsync(w.stage_dev, 0, 4 * (size_t)batch * ld, st));
    ACE_HIP(hipMemsetAsync(w.status_dev, 0, 4 * (size_t)batch, st));
    const std::vector<std::vector<int>>& rows = P.rows;
    if (d.part) {   // the full A's operators serve every restart's stages and the refinement
        w.Lf.A = w.An;
        ACE_TRY(linops_setup(w.Lf, batch, st));
    }
    auto restart = [&](int i, RestartWs& rw, hipStream_t s) -> int {
        return d.part ? run_restart_part(i, d, w.Lf, w.An, w.Bn, P.prow[i], P.pmask[i], base, rw, w.stage_dev, s)
                      : run_restart(i, d, A, w.anorm, w.Bn, rows[i], base, rw, w.stage_dev, s);
    };
    // ---- :79-83 best of restarts (A2only; the nuclear pipeline keeps the last X), in restart order
    auto take_restart = [&](int i, RestartWs& rw) -> int {
        if (cfg->variant == ACE_VARIANT_A2ONLY) {
            launch_keep_best(n, d.mt, batch, i == 0, rw.q, w.qmax, rw.X2, rw.Y2, w.Xmax, w.Ymax, st);
        } else {
            ACE_HIP(hipMemcpyAsync(w.Xmax, rw.X2, 16 * (size_t)batch * n, hipMemcpyDeviceToDevice, st));
            ACE_HIP(hipMemcpyAsync(w.Ymax, rw.Y2, 16 * (size_t)batch * d.mt, hipMemcpyDeviceToDevice, st));
        }
        ACE_HIP(hipMemcpyAsync(w.qlast, rw.q, 8 * (size_t)batch, hipMemcpyDeviceToDevice, st));
        ACE_HIP(hipMemcpyAsync(w.rank_one, rw.rank_one, batch, hipMemcpyDeviceToDevice, st));
        launch_put_col(batch, rw.status_dev, nullptr, w.status_dev, 1, 0, ~0u, st);
        ACE_LAUNCHED("refinement");
        return ACE_OK;
    };
    if (w.nrw == 1 || g_prof.on) {   // one after another (the kernel timer is not thread-safe)
        for (int i = 0; i < d.restarts; ++i) {
            ACE_TRY(restart(i, w.rw[0], st));
            ACE_TRY(take_restart(i, w.rw[0]));
        }
    } else {                         // concurrently, one host thread and stream each
        const int R = d.restarts;
        hipEvent_t ev0 = nullptr;
        std::vector<hipEvent_t> done(R, nullptr);
        std::vector<hipStream_t> ss(R, nullptr);
        std::vector<int> rc(R, ACE_OK);
        std::vector<std::string> err(R);
        auto cleanup = [&]() {
            for (int i = 0; i < R; ++i) {
                if (ss[i]) (void)hipStreamDestroy(ss[i]);
                if (done[i]) (void)hipEventDestroy(done[i]);
            }
            if (ev0) (void)hipEventDestroy(ev0);
        };
        hipError_t e = hipEventCreateWithFlags(&ev0, hipEventDisableTiming);
        for (int i = 0; i < R && e == hipSuccess; ++i) {
            e = hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&done[i], hipEventDisableTiming);
        }
        if (e == hipSuccess) e = hipEventRecord(ev0, st);   // the normalisation is done
        if (e != hipSuccess) {
            cleanup();
            return fail(ACE_ERR_HIP, "restart streams: %s", hipGetErrorString(e));
        }
        int dev = 0;
        (void)hipGetDevice(&dev);   // (the current device is per thread)
        std::vector<std::thread> th;
        for (int i = 0; i < R; ++i)
            th.emplace_back([&, i]() {
                hipError_t ei = hipSetDevice(dev);
                if (ei == hipSuccess) ei = hipStreamWaitEvent(ss[i], ev0, 0);
                rc[i] = ei == hipSuccess ? restart(i, w.rw[i], ss[i])
                                         : fail(ACE_ERR_HIP, "hipStreamWaitEvent: %s", hipGetErrorString(ei));
                if (rc[i] == ACE_OK && (ei = hipEventRecord(done[i], ss[i])) != hipSuccess)
                    rc[i] = fail(ACE_ERR_HIP, "hipEventRecord: %s", hipGetErrorString(ei));
                err[i] = g_err;
            });
        for (auto& t : th) t.join();
        for (int i = 0; i < R; ++i)
            if (rc[i] != ACE_OK) {
                for (int k = 0; k < R; ++k) (void)hipStreamSynchronize(ss[k]);
                cleanup();
                g_err = err[i];
                return rc[i];
            }
        for (int i = 0; i < R; ++i) e = e == hipSuccess ? hipStreamWaitEvent(st, done[i], 0) : e;
        if (e != hipSuccess) {
            for (int k = 0; k < R; ++k) (void)hipStreamSynchronize(ss[k]);
            cleanup();
            return fail(ACE_ERR_HIP, "hipStreamWaitEvent: %s", hipGetErrorString(e));
        }
        int rct = ACE_OK;
        for (int i = 0; i < R && rct == ACE_OK; ++i) rct = take_restart(i, w.rw[i]);
        cleanup();   // (streams and events are released once their queued work has completed)
        ACE_TRY(rct);
    }

    // the refinement's profile (:92/:100: the last restart's use_rank_one), reported per realisation
    if (cfg->variant == ACE_VARIANT_A2ONLY) launch_flag_bits(batch, w.rank_one, w.status_dev, ACE_ST_RANK_ONE, st);
    if (cfg->stop_before_refine) {   // X_max and Y_max (on the train rows), rescaled; no rollback test
        launch_fill(batch, -1.0, w.rw[0].q_s, st);
        ACE_HIP(hipMemsetAsync(w.Yr, 0, 16 * (size_t)batch * m, st));
        ACE_HIP(hipMemcpy2DAsync(w.Yr, 16 * (size_t)m, w.Ymax, 16 * (size_t)d.mt, 16 * (size_t)d.mt, batch,
                                 hipMemcpyDeviceToDevice, st));
        launch_finish(n, m, d.mt, batch, w.rw[0].q_s, w.Xmax, w.Yr, w.Xmax, w.Ymax, w.anorm, w.bnorm, Xo, Yo, nullptr, st);
        if (quality) ACE_HIP(hipMemcpyAsync(quality, w.qlast, 8 * (size_t)batch, hipMemcpyDeviceToDevice, st));
        if (stage_iters)
            ACE_HIP(hipMemcpyAsync(stage_iters, w.stage_dev, 4 * (size_t)batch * ld, hipMemcpyDeviceToDevice, st));
        if (status) ACE_HIP(hipMemcpyAsync(status, w.status_dev, 4 * (size_t)batch, hipMemcpyDeviceToDevice, st));
        ACE_LAUNCHED("pipeline outputs");
        return ACE_OK;
    }
    // ---- :89-101 refinement on the full A, r = 1, the last restart's use_rank_one
    if (!d.part) {
        w.Lf.A = w.An;
        ACE_TRY(linops_setup(w.Lf, batch, st));
    }
    AdmmParams p = base;
    p.r = 1;
    p.row_mode = 1;
    p.rank_one = w.rank_one;
    ACE_TRY(admm_run(w.Lf, p, w.s1, batch, w.Bn, w.Xmax, w.Xr, w.Yr, w.iters, (uint32_t*)w.stat, nullptr, st));
    launch_put_col(batch, w.iters, nullptr, w.stage_dev, ld, ld - 1, 0, st);
    launch_put_col(batch, w.stat, nullptr, w.status_dev, 1, 0, ~0u, st);
    // ---- :93-107 rollback and rescale
    launch_finish(n, m, d.mt, batch, w.qlast, w.Xr, w.Yr, w.Xmax, w.Ymax, w.anorm, w.bnorm, Xo, Yo,
                  (uint32_t*)w.status_dev, st);
    if (quality) ACE_HIP(hipMemcpyAsync(quality, w.qlast, 8 * (size_t)batch, hipMemcpyDeviceToDevice, st));
    if (stage_iters)
        ACE_HIP(hipMemcpyAsync(stage_iters, w.stage_dev, 4 * (size_t)batch * ld, hipMemcpyDeviceToDevice, st));
    if (status) ACE_HIP(hipMemcpyAsync(status, w.status_dev, 4 * (size_t)batch, hipMemcpyDeviceToDevice, st));
    ACE_LAUNCHED("pipeline outputs");
    return ACE_OK;
}

int ace_pipeline_solve_host(const ace_pipeline_cfg* cfg, int batch, int m, int n, int tx, int rx, const double* A,
                            const double* B, const int32_t* train_idx, double* X, double* Y, double* quality,
                            int32_t* stage_iters, uint32_t* status) {
    g_err.clear();
    PipeDims d;
    ACE_TRY(validate(cfg, batch, m, n, tx, rx, &d));
    const int ld = 4 * d.restarts + 1;
    const size_t nA = (size_t)m * n * 16, nB = (size_t)batch * m * 8, nX = (size_t)batch * n * 16,
                 nY = (size_t)batch * m * 16, ws = ace_pipeline_workspace_size(cfg, batch, m, n);
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
    void *dA, *dB, *dX, *dY, *dQ, *dI, *dS, *dW;
    hipError_t e;
    if ((e = dalloc(nA, &dA)) || (e = dalloc(nB, &dB)) || (e = dalloc(nX, &dX)) || (e = dalloc(nY, &dY)) ||
        (e = dalloc(8 * (size_t)batch, &dQ)) || (e = dalloc(4 * (size_t)batch * ld, &dI)) ||
        (e = dalloc(4 * (size_t)batch, &dS)) || (e = dalloc(ws, &dW))) {
        cleanup();
        return fail(ACE_ERR_HIP, "hipMalloc: %s", hipGetErrorString(e));
    }
    int rc = ACE_OK;
    if ((e = hipMemcpy(dA, A, nA, hipMemcpyHostToDevice)) || (e = hipMemcpy(dB, B, nB, hipMemcpyHostToDevice))) {
        cleanup();
        return fail(ACE_ERR_HIP, "hipMemcpy: %s", hipGetErrorString(e));
    }
    rc = ace_pipeline_solve_batch(cfg, batch, m, n, tx, rx, (const double*)dA, (const double*)dB, train_idx,
                                  (double*)dX, (double*)dY, (double*)dQ, (int32_t*)dI, (uint32_t*)dS, dW, ws, nullptr);
    if (rc == ACE_OK) {
        if ((e = hipDeviceSynchronize()) || (e = hipMemcpy(X, dX, nX, hipMemcpyDeviceToHost)) ||
            (e = hipMemcpy(Y, dY, nY, hipMemcpyDeviceToHost)) ||
            (quality && (e = hipMemcpy(quality, dQ, 8 * (size_t)batch, hipMemcpyDeviceToHost))) ||
            (stage_iters && (e = hipMemcpy(stage_iters, dI, 4 * (size_t)batch * ld, hipMemcpyDeviceToHost))) ||
            (status && (e = hipMemcpy(status, dS, 4 * (size_t)batch, hipMemcpyDeviceToHost))))
            rc = fail(ACE_ERR_HIP, "pipeline: %s", hipGetErrorString(e));
    }
    const std::string keep = g_err;
    cleanup();
    g_err = keep;
    return rc;
}

}  // extern "C"
