// Exact-integer applies of a phase-code sensing matrix on the int8 matrix cores
// (v_mfma_i32_32x32x32_i8), for the r = 1 ADMM iteration with one shared codebook:
//
//   apply_A   T = S - A V        S = Y - M/mu,  V = Z - N/mu   (ArgMinX residual, :325-330)
//   apply_AH  X = V + A^H g                                    (ArgMinX, :325)
//
// The codebooks of the reference are phase codes: random_probe_cb_*.mat and
// Random_Phase_State hold entries in {+-1, +-j} (times one common factor after the
// normalisation of inferLowRankV4_multi.m:27-38), the multiresolution codebooks add
// switched-off antennas (0).  Every real component of such an A is in {0, +-c}.  Then
//
//   A v = c (P + jQ)(v_r + j v_i),  P, Q in {-1, 0, 1}^(m x n)
//
// is an integer combination of the entries of v.  Each realisation's vector is cut into
// fixed-point digits against one power-of-two exponent 2^e >= max|component| (the
// Ozaki scheme): w = rint(v 2^(54-e)) is a 56-bit integer, written as seven unsigned
// 7-bit digits and a signed top digit, w = sum_t u_t 128^t.  The 2x2 real expansion of
// P + jQ times every digit plane is an exact int8 x int8 -> int32 product (|partial| <=
// 127 * 2n < 2^31), and the planes are recombined in f64 (Horner, most significant
// first).  The only rounding beyond the f64 epilogue is the truncation of v to 2^(e-55),
// i.e. the result carries an f64 GEMM's accuracy (relative error ~1e-16 of max|v|).
//
// GEMM shape: rows = (realisation, digit) pairs, 16 realisations x 8 digits = 128 rows
// per work-group; cols = output reals (512 per work-group, 8 waves x 2 tiles of 32);
// K = 2 x (complex inner dimension), staged 128 reals at a time.  The digit planes are
// formed while staging (f64 -> int digits in VGPRs -> LDS); the int8 codebook is read
// in fragment order straight from global memory (1 KiB per wave per tile and K-step,
// coalesced) two K-steps ahead.  A 32-row MFMA tile holds 4 realisations x 8 digits,
// arranged so that each lane's accumulator registers 0..7 / 8..15 are the 8 digit planes
// of one realisation at one output column: the recombination needs no data movement.
//
// Exponents: apply_A takes max|V| from the Z-step (RealState::vbound, a rigorous upper
// bound |Z| + |N|/mu formed as Z and N are written); apply_AH takes max|g| over the
// realisation's m entries in a pre-pass.  A non-finite bound yields NaN outputs for that
// realisation (the f64 product would not be finite either).
#include "ace_i8.hpp"
#include "ace_zcommon.hpp"

namespace ace {

namespace {

// Phase timestamps of work-group 5 (diagnostic build only: -DACE_PHASE_STAMPS)
#ifdef ACE_PHASE_STAMPS
#define STAMP_DECL unsigned long long ts_[12] = {}
#define STAMP(i) do { if (blockIdx.x == 5 && threadIdx.x == 0) ts_[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define STAMP_D(i) (i < k_ ? ts_[i] - ts_[i - 1] : 0ull)
#define STAMP_PRINT(name, k) do { if (blockIdx.x == 5 && threadIdx.x == 0) { const int k_ = (k); \
    printf("%s %llu %llu %llu %llu %llu %llu %llu\n", name, STAMP_D(1), STAMP_D(2), STAMP_D(3), STAMP_D(4), \
           STAMP_D(5), STAMP_D(6), STAMP_D(7)); } } while (0)
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_PRINT(name, k)
#endif

constexpr int RB = 16;           // realisations per work-group
constexpr int ROWS = RB * 8;     // MFMA rows per work-group (realisation, digit)
constexpr int KC = 128;          // K padding granule (reals) and apply_AH's staging block
constexpr int NCB = 512;         // output reals per work-group
constexpr int NT = 512;          // threads (8 waves)
constexpr int KSC = KC / 32;     // MFMA K-steps per granule

__device__ __forceinline__ int i8_nks_dev(int kc) { return (2 * kc + KC - 1) / KC * KSC; }

// Fixed-point digits of 2 complex entries (4 reals) as 8 packed dwords (byte i = real i).
__device__ __forceinline__ void digits4(const double (&v)[4], double p2, uint32_t (&out)[8]) {
    uint32_t lo[4];
    int32_t hi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double x = rint(v[i] * p2);             // |x| < 2^55 (2^54 nominal)
        const double h = floor(x * 0x1p-32);
        const double l = fma(-h, 0x1p32, x);          // [0, 2^32), exact
        hi[i] = (int32_t)h;
        lo[i] = (uint32_t)l;
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        uint32_t d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (t < 4) d[i] = (lo[i] >> (7 * t)) & 127u;
            else if (t == 4) d[i] = __builtin_amdgcn_alignbit((uint32_t)hi[i], lo[i], 28) & 127u;
            else if (t == 5) d[i] = ((uint32_t)hi[i] >> 3) & 127u;
            else if (t == 6) d[i] = ((uint32_t)hi[i] >> 10) & 127u;
            else d[i] = (uint32_t)(hi[i] >> 17) & 255u;   // signed top digit
        }
        out[t] = d[0] | (d[1] << 8) | (d[2] << 16) | (d[3] << 24);
    }
}

// A fragments of one K-step from the LDS digit image: rows 32R + (lane & 31), k bytes
// 16 (lane >> 5) .. +15 of the step.
__device__ __forceinline__ void aload(const int8_t* arow, int rstride, i4v (&af)[4]) {
#ifdef ACE_I8_PROBE_NO_LDS
    for (int R = 0; R < 4; ++R) af[R] = i4v{R, 1, 2, 3};
#else
#pragma unroll
    for (int R = 0; R < 4; ++R) af[R] = *reinterpret_cast<const i4v*>(arow + 32 * R * rstride);
#endif
}
// The 4 x 2 MFMA tiles of a wave for one K-step (codebook fragments b0, b1).
__device__ __forceinline__ void kstep(const i4v (&af)[4], i4v b0, i4v b1, i16v (&acc)[4][2]) {
#pragma unroll
    for (int R = 0; R < 4; ++R) {
        acc[R][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[R], b0, acc[R][0], 0, 0, 0);
        acc[R][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[R], b1, acc[R][1], 0, 0, 0);
    }
}

// ---- software pipeline shared by both applies.  A "stage" is SK = 2 MFMA K-steps (64 K
// reals).  Global loads are issued only at stage starts, in a fixed order, into register
// sets whose roles alternate between even and odd stages (the stage loop is unrolled by 2),
// so no register that a load is still filling is ever copied and the compiler's vmcnt
// waits are exact: a stage's codebook fragments are loaded one stage ahead, apply_A's f64
// inputs two stages ahead.  (vmcnt retires in order on CDNA; a copy of an in-flight
// register, or a load under a branch, turns every wait into vmcnt(0).)
constexpr int SK = 2;
struct BSet {
    i4v f[SK][2];
};
// codebook fragments of K-steps ks0, ks0 + 1 for this wave's two column tiles (clamped to
// the last step past the end: the loads stay unconditional)
__device__ __forceinline__ void bload(BSet& b, const i4v* bp0, const i4v* bp1, int ks0, int kmax) {
#pragma unroll
    for (int kk = 0; kk < SK; ++kk) {
        const long long ks = min(ks0 + kk, kmax);
        b.f[kk][0] = bp0[ks * 64];
        b.f[kk][1] = bp1[ks * 64];
    }
}
// SK K-steps on the digit image at arow (A fragments double-buffered one step ahead)
__device__ __forceinline__ void stage_mma(const int8_t* arow, int rstride, const BSet& b, i16v (&acc)[4][2]) {
    i4v a0[4], a1[4];
    aload(arow, rstride, a0);
    aload(arow + 32, rstride, a1);
    kstep(a0, b.f[0][0], b.f[0][1], acc);
    kstep(a1, b.f[1][0], b.f[1][1], acc);
}
// apply_A:  T = (Y - M/mu) - c A V,  V = Z - N/mu  (K = n complex, outputs m complex).
constexpr int SKR = SK * 32;       // K reals per stage
constexpr int RSA = SKR + 16;      // LDS row stride of a stage image (bytes): conflict-free b128 reads
// The body of one 16-realisation block (blockIdx-free): A8 = 2 x ROWS x RSA bytes of LDS, the four
// per-realisation scratch arrays in LDS (avok_s filled by the caller).  TOL: T goes to LDS rows
// of ldt doubles (gyk_kernel) instead of the global [nb][2 Mc] array.
template <bool TOL>
__device__ __forceinline__ void i8a_block(int nb, int Kc, int Mc, int nks, const i4v* __restrict__ Bf,
                                          const double* __restrict__ Zp, const double* __restrict__ Np,
                                          const double* __restrict__ Yp, const double* __restrict__ Mp,
                                          double* __restrict__ Tp, int ldt, const double* __restrict__ cptr,
                                          const RealState* __restrict__ rs, const double* __restrict__ zeros,
                                          const double* __restrict__ AXp, int8_t (*As)[ROWS * RSA], double* sc_s,
                                          double* imu_s, int* live_s, const int* avok_s, int j0, int cb, int rc = 1) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int bl = t >> 5, cq = t & 31, jb = j0 + bl;   // staging role: vector bl, entry 32 s + cq
    // vector jb belongs to realisation jb / rc (rc columns per realisation: the r-column stages)
    const RealState* rj = rs + (jb < nb ? jb / rc : 0);
    const bool live = jb < nb && !rj->done;
    const double imu = live ? 1.0 / rj->mu : 0.0;
    const d2* z = reinterpret_cast<const d2*>(Zp) + (long long)(live ? jb : 0) * Kc;
    const d2* nn = (live && rj->nzero) ? reinterpret_cast<const d2*>(zeros)
                                       : reinterpret_cast<const d2*>(Np) + (long long)(live ? jb : 0) * Kc;
    double p2, sc;
    plane_scale(live ? rj->vbound : 0.0, *cptr, p2, sc);
    if (cq == 0) {
        sc_s[bl] = sc;
        imu_s[bl] = imu;
        live_s[bl] = live;
    }
    const int nstage = nks / SK, kmax = nks - 1;
    struct Raw {
        d2 z, n;
    };
    auto gload = [&](int s, Raw& r) {   // unconditional (clamped) loads; masked at the digit step
        const int k = min(32 * s + cq, Kc - 1);
        r.z = z[k];
        r.n = nn[k];
    };
    auto lstore = [&](const Raw& r, int s, int buf) {
        const bool in = live && 32 * s + cq < Kc;
        const double v[2] = {in ? fma(-r.n.x, imu, r.z.x) : 0.0, in ? fma(-r.n.y, imu, r.z.y) : 0.0};
        uint32_t lo[2];
        int32_t hi[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const double x = rint(v[i] * p2);
            const double h = floor(x * 0x1p-32);
            hi[i] = (int32_t)h;
            lo[i] = (uint32_t)fma(-h, 0x1p32, x);
        }
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) {
            uint32_t d[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                if (tt < 4) d[i] = (lo[i] >> (7 * tt)) & 127u;
                else if (tt == 4) d[i] = __builtin_amdgcn_alignbit((uint32_t)hi[i], lo[i], 28) & 127u;
                else if (tt == 5) d[i] = ((uint32_t)hi[i] >> 3) & 127u;
                else if (tt == 6) d[i] = ((uint32_t)hi[i] >> 10) & 127u;
                else d[i] = (uint32_t)(hi[i] >> 17) & 255u;
            }
            *reinterpret_cast<uint16_t*>(&As[buf][lds_row(bl, tt) * RSA + 2 * cq]) = (uint16_t)(d[0] | (d[1] << 8));
        }
    };

    const int ct0 = cb * (NCB / 32) + 2 * w;   // this wave's two 32-column tiles
    const i4v* bp0 = Bf + (long long)ct0 * nks * 64 + lane;
    const i4v* bp1 = bp0 + (long long)nks * 64;

    i16v acc[4][2];
#pragma unroll
    for (int R = 0; R < 4; ++R) acc[R][0] = acc[R][1] = i16v{};

    Raw r0, r1;
    BSet bA, bB;
    bload(bA, bp0, bp1, 0, kmax);
    gload(0, r0);
    gload(1, r1);
    lstore(r0, 0, 0);
    __syncthreads();
    const int8_t* arow0 = &As[0][(lane & 31) * RSA + 16 * (lane >> 5)];
    const int8_t* arow1 = arow0 + ROWS * RSA;
    for (int s = 0; s < nstage; s += 2) {
        // even stage s: digits in buffer 0, codebook bA, raw(s + 1) in r1
        bload(bB, bp0, bp1, (s + 1) * SK, kmax);
        gload(min(s + 2, nstage - 1), r0);
        __builtin_amdgcn_sched_barrier(0);   // keep the loads at the stage start
        stage_mma(arow0, RSA, bA, acc);
        __builtin_amdgcn_sched_barrier(0);
        lstore(r1, s + 1, 1);
        __syncthreads();
        // odd stage s + 1: buffer 1, bB, raw(s + 2) in r0
        bload(bA, bp0, bp1, (s + 2) * SK, kmax);
        gload(min(s + 3, nstage - 1), r1);
        __builtin_amdgcn_sched_barrier(0);
        stage_mma(arow1, RSA, bB, acc);
        __builtin_amdgcn_sched_barrier(0);
        lstore(r0, s + 2, 0);
        __syncthreads();
    }

    // epilogue: lane (col = lane & 31, h = lane >> 5), registers 8q..8q+7 = digit planes of
    // realisation 4R + 2q + h
    const int h = lane >> 5, ldo = 2 * Mc;
#pragma unroll
    for (int R = 0; R < 4; ++R)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int blo = 4 * R + 2 * q + h, j = j0 + blo;
            if (j >= nb || !live_s[blo]) continue;
            const double scb = sc_s[blo], im = imu_s[blo];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int col = (ct0 + c) * 32 + (lane & 31);
                if (col >= ldo) continue;
                const long long off = (long long)j * ldo + col;
                // a realisation with RealState::avok takes A V = AX in any block
                const double av = avok_s[blo] ? AXp[off] : scb * recombine(acc[R][c], q);
                const double tv = fma(-Mp[off], im, Yp[off]) - av;
                if (TOL) Tp[blo * ldt + col] = tv;
                else Tp[off] = tv;
            }
        }
}

__global__ __launch_bounds__(NT, 1) void i8a_kernel(int nb, int Kc, int Mc, int nks, const i4v* __restrict__ Bf,
                                                    const double* __restrict__ Zp, const double* __restrict__ Np,
                                                    const double* __restrict__ Yp, const double* __restrict__ Mp,
                                                    double* __restrict__ Tp, const double* __restrict__ cptr,
                                                    const RealState* __restrict__ rs, const double* __restrict__ zeros,
                                                    const double* __restrict__ AXp, int rc) {
    __shared__ __attribute__((aligned(16))) int8_t As[2][ROWS * RSA];
    __shared__ double sc_s[RB], imu_s[RB];
    __shared__ int live_s[RB], avok_s[RB];
    const int t = threadIdx.x, j0 = blockIdx.x * RB;
    if (t < RB) {   // per vector (the result never depends on the block it shares)
        const int j = j0 + t;
        avok_s[t] = AXp && j < nb && !rs[j].done && rs[j].avok;   // (r = 1 only: AXp is null otherwise)
    }
    __syncthreads();
    i8a_block<false>(nb, Kc, Mc, nks, Bf, Zp, Np, Yp, Mp, Tp, 0, cptr, rs, zeros, AXp, As, sc_s, imu_s, live_s, avok_s,
                     j0, blockIdx.y, rc);
}

// apply_AH in the Z-step's wmode:  W = c A^H g  (K = m complex, outputs n complex).
// The digit planes of all of K stay in LDS (dynamic, ROWS x (32 nks + 16) bytes) and the
// work-group sweeps every 512-column block of the output as one flat sequence of K-steps,
// so the exponent pre-pass and the staging run once per 16 realisations and the codebook
// pipeline runs across block boundaries.
//
// KY (apply_K, KY = K Y with K = A A^H = c^2 K_int, K_int a Gaussian-integer matrix with
// |entries| <= 2n): the codebook operand holds the two base-128 digit planes of the real
// expansion of K_int, interleaved by 32-column tile (low digit, high digit) so that a wave's
// two accumulator tiles are the two planes of the same 32 output columns; they are combined
// exactly in int32 (acc_lo + 128 acc_hi) before the recombination.  A work-group then covers
// 256 output columns per block.
//
// FUSE (unit path, from r02): the steady-state Z-step's data pass runs in the epilogue.  For a
// realisation with N = 0 and a valid perturbation certificate (RealState::kfok, nzero) the
// epilogue forms X = Z + W (xw with N = 0) and stores it as Z' = E = X instead of storing W, and
// reduces ||X||^2 and ||X - Z||^2; W then never goes through HBM.  The sums go to RealState
// (fs0, fs3, fzit) and zstep1w_kernel, one wave per realisation, checks the bound and runs the
// iteration control (or, if the bound fails, the full Z-step with X read from Z').  An
// ineligible realisation gets W as before.
struct FuseState {   // per realisation, loaded in the prologue
    int el, keep_cur, optsrc;
};
// The block body.  Ad: the digit planes (ROWS x (32 nks + 16) bytes of LDS); zsum (FUSE): the
// per-lane partial sums ||X||^2, ||X - Z||^2 of each (wave, realisation pair slot), one slot per
// lane accumulated over the column blocks (no shuffles in the epilogue), [8 waves][8 (R, q)][2]
// [64 lanes] doubles = 64 KiB.  gl (GLDS): g of the block's realisations in LDS rows of gst
// complex (the fused g / Y-step / apply_AH kernel), instead of Gp in global memory.
template <bool KY, bool FUSE, bool GLDS>
__device__ __forceinline__ void i8ah_body(int nb, int Kc, int Mc, int nks, const i4v* __restrict__ Bf,
                                          const double* __restrict__ Gp, double* __restrict__ Wp,
                                          const double* __restrict__ cptr, const RealState* __restrict__ rs,
                                          const ZArgs& za, int8_t* Ad, double* zsum, const d2* gl, int gst) {
    __shared__ double sc_s[RB], imu_s[RB];
    __shared__ int live_s[RB];
    __shared__ FuseState fs_s[FUSE ? RB : 1];
    __shared__ int z0_s[(!FUSE && !KY) ? RB : 1];
    __shared__ int nz_s[(!FUSE && !KY) ? RB : 1];   // (xzn, r-column stages: N held as exact zero, RealState::nzero)
    const int rst = 32 * nks + 16;   // LDS row stride (bytes)

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int j0 = blockIdx.x * RB;
    const int bl = t >> 5, cp = t & 31, jb = j0 + bl;
    STAMP_DECL;
    STAMP(0);
    // m-space realisations (RealState::mzit, set by gyk_body of this launch) need no pass; the
    // matz launch (launch_i8_msp_optx) takes exactly the realisations with opt_X in m-space form
    const bool matz = !FUSE && !KY && za.matz;
    // r-column stages (za.r > 1, !FUSE): vector jb belongs to realisation jb / r
    const int rc = (!FUSE && za.r > 1) ? za.r : 1;
    const bool live = jb < nb && (matz ? rs[jb].optsrc == 3
                                       : (!rs[jb / rc].done && !(za.msp && rs[jb / rc].mzit == za.it)));
    // a block none of whose realisations needs the pass (all settled in m-space, done, or past nb)
    // skips it whole (uniform across the work-group)
    if (!__syncthreads_or(live)) return;
    const int zn_id = 1 + (za.it & 1);
    if constexpr (!FUSE && !KY) {
        if (matz && t < RB) z0_s[t] = j0 + t < nb ? rs[j0 + t].z0id : 0;
    }
    if constexpr (FUSE) {
        if (t < RB) {
            const int j = j0 + t;
            FuseState f{};
            if (j < nb && !rs[j].done && !(za.msp && rs[j].mzit == za.it)) {
                const RealState& r = rs[j];
                f.el = r.kfok && r.nzero;
                const bool improved_pre = sqrt(r.obj2) < r.opt_obj;   // (as the Z-step decides it)
                f.keep_cur = !improved_pre && !(r.opt_obj < INFINITY);
                f.optsrc = r.optsrc;
            }
            fs_s[t] = f;
        }
    }
    const d2* g = reinterpret_cast<const d2*>(Gp) + (long long)jb * Kc;

    // g of this realisation: 2 complex entries per 128-real block per thread, one batch of
    // loads (up to GR blocks held in registers; longer K re-reads the rest from L2)
    constexpr int GR = 4;
    const int nst = nks / 4;
    d2 gv[GR][2];
    double mx = 0.0, sn = 0.0;   // max |g| of the realisation over this half-wave
    auto gat = [&](int s, int u) -> d2 {
        const int k = 64 * s + 2 * cp + u;
        if constexpr (GLDS) return (live && k < Kc) ? gl[bl * gst + k] : make_double2(0.0, 0.0);
        return (live && k < Kc) ? g[k] : make_double2(0.0, 0.0);
    };
#pragma unroll
    for (int s = 0; s < GR; ++s)
#pragma unroll
        for (int u = 0; u < 2; ++u) gv[s][u] = s < nst ? gat(s, u) : make_double2(0.0, 0.0);
    auto acc_max = [&](d2 v) {
        const double ax = fabs(v.x), ay = fabs(v.y);
        mx = fmax(mx, fmax(ax, ay));
        sn += 0.0 * (ax + ay);   // NaN / Inf sticky
    };
#pragma unroll
    for (int s = 0; s < GR; ++s) {
        acc_max(gv[s][0]);
        acc_max(gv[s][1]);
    }
    for (int s = GR; s < nst; ++s) {
        acc_max(gat(s, 0));
        acc_max(gat(s, 1));
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
        mx = fmax(mx, __shfl_xor(mx, o, 64));
        sn += __shfl_xor(sn, o, 64);
    }
    double p2, sc;
    plane_scale(mx + sn, *cptr, p2, sc);
    if (cp == 0) {
        sc_s[bl] = sc;
        live_s[bl] = live;
        imu_s[bl] = (!KY && !FUSE && za.xzn && live) ? 1.0 / rs[jb / rc].mu : 0.0;
        if constexpr (!FUSE && !KY) nz_s[bl] = za.xzn && live && rc > 1 && rs[jb / rc].nzero;
    }
    for (int s = 0; s < nst; ++s) {
        d2 x0, x1;
        if (s < GR) {
#pragma unroll
            for (int q = 0; q < GR; ++q)
                if (q == s) {
                    x0 = gv[q][0];
                    x1 = gv[q][1];
                }
        } else {
            x0 = gat(s, 0);
            x1 = gat(s, 1);
        }
        const double v[4] = {x0.x, x0.y, x1.x, x1.y};
        uint32_t d[8];
        digits4(v, p2, d);
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) *reinterpret_cast<uint32_t*>(&Ad[lds_row(bl, tt) * rst + KC * s + 4 * cp]) = d[tt];
    }
    __syncthreads();
    STAMP(1);
    if constexpr (FUSE) {
        // deferred opt_X: the Z' buffer of an eligible realisation holds its best iterate -- keep
        // it before the epilogue overwrites it (rare; fs_s is visible after the staging barrier)
        for (int r = 0; r < RB; ++r)
            if (fs_s[r].el && fs_s[r].optsrc == zn_id) {
                const long long o = (long long)(j0 + r) * 2 * Mc;
                for (int i = t; i < 2 * Mc; i += NT) za.optX[o + i] = za.Zn[o + i];
                __syncthreads();
                if (t == 0) za.st[j0 + r].optsrc = 0;
            }
    }

    const int h = lane >> 5, ldo = 2 * Mc, ocb = KY ? NCB / 2 : NCB, ncb = (ldo + ocb - 1) / ocb;
    const int8_t* arow = &Ad[(lane & 31) * rst + 16 * (lane >> 5)];
    const int total = ncb * nks;   // flat (column block, K-step) sequence, a multiple of 2 SK
    auto bfl = [&](BSet& b, int f0) {   // codebook fragments of flat steps f0, f0 + 1 (clamped)
#pragma unroll
        for (int kk = 0; kk < SK; ++kk) {
            const int f = min(f0 + kk, total - 1), cb = f / nks, ks = f - cb * nks;
            const i4v* p = Bf + ((long long)(cb * (NCB / 32) + 2 * w) * nks + ks) * 64 + lane;
            b.f[kk][0] = p[0];
            b.f[kk][1] = p[(long long)nks * 64];
        }
    };
    // FUSE: Z at this lane's 16 epilogue outputs of block cbk (eligible realisations)
    auto zload = [&](int cbk, double (&zv)[4][2][2]) {
        const int ct0 = cbk * (NCB / 32) + 2 * w;
#pragma unroll
        for (int R = 0; R < 4; ++R)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int blo = 4 * R + 2 * q + (lane >> 5), j = min(j0 + blo, nb - 1);
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const int col = min((ct0 + c) * 32 + (lane & 31), 2 * Mc - 1);
                    zv[R][q][c] = fs_s[blo].el ? za.Z[(long long)j * 2 * Mc + col] : 0.0;
                }
            }
    };
    auto epilogue = [&](int cbk, i16v (&acc)[4][2], const double (&zv)[4][2][2]) {
        if constexpr (KY) {   // one 32-column output tile per wave: low + 128 x high digit plane
            const int col = (cbk * (NCB / 64) + w) * 32 + (lane & 31);
#pragma unroll
            for (int R = 0; R < 4; ++R)
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int blo = 4 * R + 2 * q + h, j = j0 + blo;
                    if (j >= nb || !live_s[blo] || col >= ldo) continue;
                    i16v cmb;
#pragma unroll
                    for (int e = 0; e < 16; ++e) cmb[e] = acc[R][0][e] + 128 * acc[R][1][e];
                    Wp[(long long)j * ldo + col] = sc_s[blo] * recombine(cmb, q);
                }
#pragma unroll
            for (int R = 0; R < 4; ++R) acc[R][0] = acc[R][1] = i16v{};
            return;
        }
        const int ct0 = cbk * (NCB / 32) + 2 * w;
        if constexpr (FUSE) {   // zv: requested two stages ahead by the sweep (zload)
#pragma unroll
            for (int R = 0; R < 4; ++R)
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int blo = 4 * R + 2 * q + h, j = j0 + blo;
                    const bool el = fs_s[blo].el, kc = fs_s[blo].keep_cur;
                    double p0 = 0.0, p3 = 0.0;
                    if (j < nb && live_s[blo]) {
                        const double scb = sc_s[blo];
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            const int col = (ct0 + c) * 32 + (lane & 31);
                            if (col >= ldo) continue;
                            const long long off = (long long)j * ldo + col;
                            const double wv = scb * recombine(acc[R][c], q);
                            if (el) {
                                const double x = zv[R][q][c] + wv, d = x - zv[R][q][c];
                                za.Zn[off] = x;
                                if (kc) za.Xcur[off] = x;
                                p0 += x * x;
                                p3 += d * d;
                            } else {
                                Wp[off] = wv;
                            }
                        }
                    }
                    if (el) {   // this lane's slots (fixed order over the blocks)
                        double* zs = zsum + ((w * 8 + 2 * R + q) * 2) * 64 + lane;
                        zs[0] = cbk == 0 ? p0 : zs[0] + p0;
                        zs[64] = cbk == 0 ? p3 : zs[64] + p3;
                    }
                }
        } else {
#pragma unroll
        for (int R = 0; R < 4; ++R)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int blo = 4 * R + 2 * q + h, j = j0 + blo;
                if (j >= nb || !live_s[blo]) continue;
                const double scb = sc_s[blo];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const int col = (ct0 + c) * 32 + (lane & 31);
                    if (col >= ldo) continue;
                    const long long off = (long long)j * ldo + col;
                    const double wv = scb * recombine(acc[R][c], q);
                    if (matz) Wp[off] = (z0_s[blo] == 1 ? za.Z : za.Zn)[off] + wv;   // Z0 + A^H opt_S
                    else if (za.xzn) {   // X = V + A^H g; N held as exact zero reads the zero row (no branch)
                        const double* nrow = nz_s[blo] ? za.zeros : za.N + (long long)j * ldo;
                        Wp[off] = fma(-nrow[col], imu_s[blo], za.Z[off]) + wv;
                    }
                    else Wp[off] = wv;
                }
            }
        }
#pragma unroll
        for (int R = 0; R < 4; ++R) acc[R][0] = acc[R][1] = i16v{};
    };
    i16v acc[4][2];
#pragma unroll
    for (int R = 0; R < 4; ++R) acc[R][0] = acc[R][1] = i16v{};
    BSet bA, bB;
    bfl(bA, 0);
    if constexpr (FUSE) {
        // the last loop step of every block is peeled: its Z loads go out right after the stage's
        // codebook loads, so no wait before the epilogue's own waits for them (vmcnt retires in
        // order: a load issued under a branch would make every wait a full drain)
        double zv[4][2][2];
        const int per = nks / (2 * SK);
        for (int cbk = 0; cbk < ncb; ++cbk) {
            const int f0 = cbk * nks;
            for (int i = 0; i < per - 1; ++i) {
                const int f = f0 + 2 * SK * i;
                bfl(bB, f + SK);
                __builtin_amdgcn_sched_barrier(0);
                stage_mma(arow + 32 * (f % nks), rst, bA, acc);
                __builtin_amdgcn_sched_barrier(0);
                bfl(bA, f + 2 * SK);
                __builtin_amdgcn_sched_barrier(0);
                stage_mma(arow + 32 * ((f + SK) % nks), rst, bB, acc);
                __builtin_amdgcn_sched_barrier(0);
            }
            const int f = f0 + 2 * SK * (per - 1);
            bfl(bB, f + SK);
            zload(cbk, zv);
            __builtin_amdgcn_sched_barrier(0);
            stage_mma(arow + 32 * (f % nks), rst, bA, acc);
            __builtin_amdgcn_sched_barrier(0);
            bfl(bA, f + 2 * SK);
            __builtin_amdgcn_sched_barrier(0);
            stage_mma(arow + 32 * ((f + SK) % nks), rst, bB, acc);
            __builtin_amdgcn_sched_barrier(0);
            epilogue(cbk, acc, zv);
        }
    } else {
        const double zv0[4][2][2] = {};
        for (int f = 0; f < total; f += 2 * SK) {
            bfl(bB, f + SK);
            __builtin_amdgcn_sched_barrier(0);   // keep the loads at the stage start
            stage_mma(arow + 32 * (f % nks), rst, bA, acc);
            __builtin_amdgcn_sched_barrier(0);
            bfl(bA, f + 2 * SK);
            __builtin_amdgcn_sched_barrier(0);
            stage_mma(arow + 32 * ((f + SK) % nks), rst, bB, acc);
            __builtin_amdgcn_sched_barrier(0);
            if ((f + 2 * SK) % nks == 0) epilogue(f / nks, acc, zv0);
        }
    }
    STAMP(2);
    if (!KY && !FUSE) STAMP_PRINT("i8ah prologue|sweep:", 3);
    if constexpr (!FUSE && !KY) {
        if (matz && (t & 31) == 0 && live) za.st[jb].optsrc = 0;
    }
    if constexpr (FUSE) {
        __syncthreads();
        {   // half-wave t >> 5 = realisation blo: its 8 waves x 32 lanes of slots, fixed order
            const int blo = t >> 5, sub = t & 31, R = blo >> 2, q = (blo >> 1) & 1, hh = blo & 1;
            double s0 = 0.0, s3 = 0.0;
            if (fs_s[blo].el && live_s[blo])
                for (int ww = 0; ww < 8; ++ww) {
                    const double* zs = zsum + ((ww * 8 + 2 * R + q) * 2) * 64 + 32 * hh + sub;
                    s0 += zs[0];
                    s3 += zs[64];
                }
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) {
                s0 += __shfl_xor(s0, o, 64);
                s3 += __shfl_xor(s3, o, 64);
            }
            if (sub == 0 && fs_s[blo].el && live_s[blo]) {
                RealState* st = za.st + j0 + blo;
                st->fs0 = s0;   // ||E||^2 = ||X||^2
                st->fs3 = s3;   // ||E - E_prev||^2 = ||X - Z||^2
                st->fzit = za.it;
            }
        }
        STAMP(3);
        STAMP_PRINT("i8ah-fused prologue|sweep|post:", 4);
    }
}
template <bool KY, bool FUSE>
__global__ __launch_bounds__(NT, 1) void i8ah_kernel(int nb, int Kc, int Mc, int nks, const i4v* __restrict__ Bf,
                                                     const double* __restrict__ Gp, double* __restrict__ Wp,
                                                     const double* __restrict__ cptr,
                                                     const RealState* __restrict__ rs, ZArgs za) {
    extern __shared__ __attribute__((aligned(16))) int8_t Ad[];
    double* zsum = reinterpret_cast<double*>(Ad + ((ROWS * (32 * nks + 16) + 255) & ~255));
    i8ah_body<KY, FUSE, false>(nb, Kc, Mc, nks, Bf, Gp, Wp, cptr, rs, za, Ad, zsum, nullptr, 0);
}

// Codebook check and expansion.  cmax = max |component| of A (device scalar).  Each
// complex entry A[i][k] = c (p + j q) must have p, q in {-1, 0, 1}; flag is set otherwise.
//   apply_A  (cols 2m, K 2n):  L[2i][2k] = p, L[2i][2k+1] = -q, L[2i+1][2k] = q, L[2i+1][2k+1] = p
//   apply_AH (cols 2n, K 2m):  H[2k][2i] = p, H[2k][2i+1] = q, H[2k+1][2i] = -q, H[2k+1][2i+1] = p
// Fragment order: byte (col, k) of a [cols][K] matrix at ((col/32 * nks + k/32) * 64 + col%32 +
// 32 ((k%32)/16)) * 16 + k%16  (lane l of an MFMA operand holds col l&31, k 16 (l>>5) .. +15).
__device__ __forceinline__ long long frag_off(int col, int k, int nks) {
    return ((long long)((col >> 5) * nks + (k >> 5)) * 64 + (col & 31) + 32 * ((k & 31) >> 4)) * 16 + (k & 15);
}
__global__ __launch_bounds__(256) void i8_expand_kernel(int m, int n, const double* __restrict__ Ap,
                                                         const double* __restrict__ cmax, int8_t* __restrict__ LA,
                                                         int nksA, int8_t* __restrict__ LH, int nksH, int* flag) {
    const long long e = blockIdx.x * 256LL + threadIdx.x;
    if (e >= (long long)m * n) return;
    const int i = (int)(e / n), k = (int)(e % n);
    const d2 a = reinterpret_cast<const d2*>(Ap)[e];
    const double c = *cmax;
    auto code = [&](double x, int& ok) -> int {
        if (x == c) return 1;
        if (x == -c) return -1;
        if (x == 0.0) return 0;
        ok = 0;
        return 0;
    };
    int ok = 1;
    const int p = code(a.x, ok), q = code(a.y, ok);
    if (!ok) atomicOr(flag, 1);
    LA[frag_off(2 * i, 2 * k, nksA)] = (int8_t)p;
    LA[frag_off(2 * i, 2 * k + 1, nksA)] = (int8_t)(-q);
    LA[frag_off(2 * i + 1, 2 * k, nksA)] = (int8_t)q;
    LA[frag_off(2 * i + 1, 2 * k + 1, nksA)] = (int8_t)p;
    LH[frag_off(2 * k, 2 * i, nksH)] = (int8_t)p;
    LH[frag_off(2 * k, 2 * i + 1, nksH)] = (int8_t)q;
    LH[frag_off(2 * k + 1, 2 * i, nksH)] = (int8_t)(-q);
    LH[frag_off(2 * k + 1, 2 * i + 1, nksH)] = (int8_t)p;
}
// ---- fused r = 1 middle of the iteration for 16-realisation blocks (m <= GYK_MAXM):
//   g = G T on the f64 matrix cores (3M form; G streamed from L2 in fragment order, T from LDS)
//   Y-step (ArgMinY, M update, :326-337) with the five sums completed in the work-group
//   K Y_new on the int8 matrix cores (digit planes of Y_new from LDS, as i8ah_kernel<true>)
//   the dual terms dY^H (K Y - K Y0), Y^H K Y and the opt_Y copy
// so that neither the Z-step nor a separate K Y launch touches Y or K Y again.
#ifndef ACE_GSK
#define ACE_GSK 4
#endif
constexpr int GSK = ACE_GSK;          // f64 K-steps (4 complex each) per pipeline stage
constexpr int GRB = 16;         // realisations per work-group (one f64 MFMA row tile)
__host__ __device__ __forceinline__ int gyk_mp(int m) { return (m + 31) & ~31; }
struct GSet {
    d2 f[GSK][2];
};

// One output of the fused Y-step (ArgMinY with its zero guard, inferLowRankV4_multi.m:511-533, and
// the M update): g from the 3M accumulators, AX = (Y - M/mu) - g, Y', M', and the five sums plus the
// max |Y'| (with its NaN-sticky term) into v[0..6].  Shared by gyk_body and msr_kernel, so that the
// two kernels form every iterate with the same operations in the same order: no multiply-add
// contraction here (the compiler's fusion choices depend on the basic blocks around an inlined copy).
__device__ __forceinline__ void ystep_elem(double e1, double e2, double e3, double mu, d2 mii, d2 yo, double Bi,
                                           d2& gv, d2& ax, d2& mn, d2& y, double (&v)[9]) {
#pragma clang fp contract(off)
    // (written out in scalars: the pragma governs only the operations spelled here, not those of
    // the complex helpers)
    gv = make_double2(e1 - e2, e3 - e1 - e2);
    const double imu = 1.0 / mu;
    const double pr = mii.x * imu, pi = mii.y * imu;   // M / mu
    ax = make_double2((yo.x - pr) - gv.x, (yo.y - pi) - gv.y);
    double cr = ax.x + pr, ci = ax.y + pi;
    double d = sqrt(cr * cr + ci * ci);
    if (d == 0.0) {   // ArgMinY zero guard (:516-520 / :524-528)
        cr = 1.0;
        ci = 0.0;
        d = 1.0;
    }
    const double f = (Bi / d + mu) / (1.0 + mu);
    y = make_double2(cr * f, ci * f);
    const double jr = ax.x - y.x, ji = ax.y - y.y;
    mn = make_double2(mii.x + jr * mu, mii.y + ji * mu);
    const double aax = sqrt(ax.x * ax.x + ax.y * ax.y) - Bi;
    v[0] += aax * aax;
    v[1] += ax.x * ax.x + ax.y * ax.y;
    v[2] += y.x * y.x + y.y * y.y;
    v[3] += jr * jr + ji * ji;
    const double dr = y.x - yo.x, di = y.y - yo.y;
    v[4] += dr * dr + di * di;
    const double ay = fmax(fabs(y.x), fabs(y.y));
    v[5] = fmax(v[5], ay);
    v[6] += 0.0 * (fabs(y.x) + fabs(y.y));   // NaN / Inf sticky
}
// m-space sums of one output (RealState::msp): Re (A Z)^H g with A Z = A V = (Y - M/mu) - T (T's
// input), and g^H K g = Re g^H (T - g), into v[7], v[8] (no contraction, as ystep_elem)
__device__ __forceinline__ void msp_sums_elem(d2 yo, d2 mii, double imu, d2 tv, d2 gv, double (&v)[9]) {
#pragma clang fp contract(off)
    const double ar = (yo.x - mii.x * imu) - tv.x, ai = (yo.y - mii.y * imu) - tv.y;
    v[7] += ar * gv.x + ai * gv.y;
    v[8] += gv.x * (tv.x - gv.x) + gv.y * (tv.y - gv.y);
}

template <bool GLDS>   // g stays in the LDS rows of T for the fused apply_AH (gyf_kernel) instead of a.g
__device__ __forceinline__ void gyk_body(int nb, int m, const GykArgs& a, unsigned char* smem, const ZArgs& za,
                                         int za_ctl) {
    __shared__ double red[8][GRB][9];
    __shared__ double sc_s[GRB], p2_s[GRB];
    __shared__ int live_s[GRB], imp_s[GRB], avok_s[GRB], oys_s[GRB], pend_s[GRB], msp_s[GRB], ent_s[GRB], oss_s[GRB];
    __shared__ double imu0_s[GRB], mu_s[GRB];
    const int mp = gyk_mp(m), tst = mp + 1;            // LDS row stride (complex, odd)
    d2* Ts = reinterpret_cast<d2*>(smem);               // [16][tst]: T, then Y_new
    int8_t* Ad = reinterpret_cast<int8_t*>(smem) + ((GRB * tst * 16 + 255) & ~255);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, j0 = blockIdx.x * GRB;
    STAMP_DECL;
    STAMP(0);
    // The inputs of T = (Y - M/mu) - AX (the steady state: every realisation has avok) are requested
    // before the realisations' state, so the two round trips overlap (unconditional, clamped
    // addresses; mp <= 256 gives at most 8 elements per thread)
    constexpr int TU = 8;
    d2 tyv[TU], tmv[TU], txv[TU];
    const bool early = a.LA && a.AX;
    if (early) {
#pragma unroll
        for (int u = 0; u < TU; ++u) {
            const int idx = min(t + NT * u, GRB * mp - 1), jl = idx / mp, k = min(idx - jl * mp, m - 1);
            const long long o = (long long)min(j0 + jl, nb - 1) * m + k;
            tyv[u] = reinterpret_cast<const d2*>(a.Yo)[o];
            tmv[u] = reinterpret_cast<const d2*>(a.M)[o];
            txv[u] = reinterpret_cast<const d2*>(a.AX)[o];
        }
    }
    if (t < GRB) {
        const int j = j0 + t;
        const bool lv = j < nb && !a.rs[j].done;
        live_s[t] = lv;
        avok_s[t] = lv && a.AX && a.rs[j].avok;
        mu_s[t] = lv ? a.rs[j].mu : 1.0;
        imu0_s[t] = lv ? 1.0 / mu_s[t] : 0.0;
        oys_s[t] = lv ? a.rs[j].optysrc : 0;
        pend_s[t] = lv && a.lazy && a.rs[j].dpend;
        // m-space step candidate (RealState::msp): certified, N = 0, V = the previous X, an opt_X
        // recorded, and the previous iteration left ||Z||^2 in fs0 (fused pass or m-space step).
        // A realisation already in the form stays in it; a new one enters after the Y-step only if
        // the bound has room (below), else it takes the fused apply_AH pass as before.
        int ms = 0, en = 0;
        if (GLDS && a.msp && lv && a.it >= 2) {
            const RealState& r = a.rs[j];
            // (Z of a realisation in the form is not in memory: it stays in it; a failed bound
            // materialises it in the Z-step)
            ms = r.msp || (avok_s[t] && r.kfok && r.nzero && r.opt_obj < INFINITY && r.fzit == a.it - 1);
            en = ms && !r.msp;
        }
        msp_s[t] = ms;
        ent_s[t] = en;
        oss_s[t] = lv ? a.rs[j].optsrc : 0;
    }
    __syncthreads();
    // T of the avok realisations from the early loads (a block that needs apply_A or finishes a
    // pending test rewrites Ts below)
    auto t_from = [&](const d2 (&yv)[TU], const d2 (&mv)[TU], const d2 (&xv)[TU]) {
#pragma unroll
        for (int u = 0; u < TU; ++u) {
            const int idx = t + NT * u;
            if (idx >= GRB * mp) continue;
            const int jl = idx / mp, k = idx - jl * mp;
            d2 v = make_double2(0.0, 0.0);
            if (live_s[jl] && avok_s[jl] && k < m) {
                const double im = imu0_s[jl];
                v = make_double2(fma(-mv[u].x, im, yv[u].x) - xv[u].x, fma(-mv[u].y, im, yv[u].y) - xv[u].y);
            }
            Ts[jl * tst + k] = v;
        }
    };
    if (early) t_from(tyv, tmv, txv);
    const int nksK = i8_nks_dev(m), rst = 32 * nksK + 16;
    // ---- lazy dual residual: the previous Z-step left some convergence tests pending (the primal
    // part held, the combined part failed: inferLowRankV4_multi.m:372 needs res_dual).  They are
    // finished here, before this iteration uses mu, from ||A^H Y_k||^2 = Y_k^H K Y_k and
    // ||A^H (Y_k - Y_{k-1})||^2 (Y_k in Yo, Y_{k-1} still in Yn) on the int8 matrix cores (two
    // passes of the K Y machinery below).  Rare: a few iterations per solve.
    if (a.lazy && __syncthreads_or(t < GRB && pend_s[t])) {
        const int bl = t >> 5, cp = t & 31, h = lane >> 5, ldo = 2 * m, ocb = NCB / 2, ncb = (ldo + ocb - 1) / ocb;
        const int8_t* arow = &Ad[(lane & 31) * rst + 16 * (lane >> 5)];
        const i4v* Bf = reinterpret_cast<const i4v*>(a.LK);
        const int total = ncb * nksK;
        const double* Ysd = reinterpret_cast<const double*>(Ts);
        for (int pass = 0; pass < 2; ++pass) {
            double mx = 0.0, sn = 0.0;
            for (int i = cp; i < mp; i += 32) {   // half-wave bl: realisation bl
                d2 v = make_double2(0.0, 0.0);
                if (pend_s[bl] && i < m) {
                    const long long o = (long long)(j0 + bl) * m + i;
                    const d2 yk = reinterpret_cast<const d2*>(a.Yo)[o];
                    v = pass ? csub(yk, reinterpret_cast<const d2*>(a.Yn)[o]) : yk;
                }
                Ts[bl * tst + i] = v;
                mx = fmax(mx, fmax(fabs(v.x), fabs(v.y)));
                sn += 0.0 * (fabs(v.x) + fabs(v.y));
            }
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) {
                mx = fmax(mx, __shfl_xor(mx, o, 64));
                sn += __shfl_xor(sn, o, 64);
            }
            double p2, sc;
            plane_scale(mx + sn, a.c8[1], p2, sc);
            if (cp == 0) sc_s[bl] = sc;
            __syncthreads();
            for (int s = 0; s < nksK / KSC; ++s) {
                d2 x[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int k = 64 * s + 2 * cp + u;
                    x[u] = k < m ? Ts[bl * tst + k] : make_double2(0.0, 0.0);
                }
                const double v[4] = {x[0].x, x[0].y, x[1].x, x[1].y};
                uint32_t d[8];
                digits4(v, p2, d);
#pragma unroll
                for (int tt = 0; tt < 8; ++tt)
                    *reinterpret_cast<uint32_t*>(&Ad[lds_row(bl, tt) * rst + KC * s + 4 * cp]) = d[tt];
            }
            __syncthreads();
            auto bfl = [&](BSet& bs, int f0) {
#pragma unroll
                for (int kk = 0; kk < SK; ++kk) {
                    const int f = min(f0 + kk, total - 1), cb = f / nksK, ks = f - cb * nksK;
                    const i4v* pp = Bf + ((long long)(cb * (NCB / 32) + 2 * w) * nksK + ks) * 64 + lane;
                    bs.f[kk][0] = pp[0];
                    bs.f[kk][1] = pp[(long long)nksK * 64];
                }
            };
            double pacc[4][2];
#pragma unroll
            for (int R = 0; R < 4; ++R) pacc[R][0] = pacc[R][1] = 0.0;
            i16v acc[4][2];
#pragma unroll
            for (int R = 0; R < 4; ++R) acc[R][0] = acc[R][1] = i16v{};
            BSet bA, bB;
            bfl(bA, 0);
            for (int f = 0; f < total; f += 2 * SK) {
                bfl(bB, f + SK);
                __builtin_amdgcn_sched_barrier(0);
                stage_mma(arow + 32 * (f % nksK), rst, bA, acc);
                __builtin_amdgcn_sched_barrier(0);
                bfl(bA, f + 2 * SK);
                __builtin_amdgcn_sched_barrier(0);
                stage_mma(arow + 32 * ((f + SK) % nksK), rst, bB, acc);
                __builtin_amdgcn_sched_barrier(0);
                if ((f + 2 * SK) % nksK == 0) {   // v^H (K v) over this 32-column tile
                    const int col = ((f / nksK) * (NCB / 64) + w) * 32 + (lane & 31);
#pragma unroll
                    for (int R = 0; R < 4; ++R)
#pragma unroll
                        for (int q = 0; q < 2; ++q) {
                            const int blo = 4 * R + 2 * q + h;
                            if (pend_s[blo] && col < ldo) {
                                i16v cmb;
#pragma unroll
                                for (int e = 0; e < 16; ++e) cmb[e] = acc[R][0][e] + 128 * acc[R][1][e];
                                pacc[R][q] += Ysd[2 * blo * tst + col] * (sc_s[blo] * recombine(cmb, q));
                            }
                        }
#pragma unroll
                    for (int R = 0; R < 4; ++R) acc[R][0] = acc[R][1] = i16v{};
                }
            }
#pragma unroll
            for (int R = 0; R < 4; ++R)
#pragma unroll
                for (int q = 0; q < 2; ++q) {
#pragma unroll
                    for (int o = 1; o < 32; o <<= 1) pacc[R][q] += __shfl_xor(pacc[R][q], o, 64);
                    if ((lane & 31) == 0) red[w][4 * R + 2 * q + h][pass] = pacc[R][q];
                }
            __syncthreads();
        }
        if (t < GRB && pend_s[t]) {
            double nv = 0.0, dv = 0.0;
            for (int q = 0; q < 8; ++q) {   // fixed order over the waves
                nv += red[q][t][0];
                dv += red[q][t][1];
            }
            RealState* rs = a.rs + j0 + t;
            if (dual_finish(a.dc, rs, dv, nv)) live_s[t] = 0;   // stopped at the previous iteration
            mu_s[t] = rs->mu;
            imu0_s[t] = 1.0 / mu_s[t];
        }
        __syncthreads();
        if (early) {   // Ts was scratch here, and mu may have changed: T again (rare)
#pragma unroll
            for (int u = 0; u < TU; ++u) {
                const int idx = min(t + NT * u, GRB * mp - 1), jl = idx / mp, k = min(idx - jl * mp, m - 1);
                const long long o = (long long)min(j0 + jl, nb - 1) * m + k;
                tyv[u] = reinterpret_cast<const d2*>(a.Yo)[o];
                tmv[u] = reinterpret_cast<const d2*>(a.M)[o];
                txv[u] = reinterpret_cast<const d2*>(a.AX)[o];
            }
            t_from(tyv, tmv, txv);
        }
    }
    // deferred opt_Y (RealState::optysrc): the best Y_new still lives in the buffer this iteration's
    // Y-step is about to overwrite -- save it first (rare: no better iterate in the last iteration)
    if (a.yn_id)
        for (int r = 0; r < GRB; ++r)
            if (oys_s[r] == a.yn_id)
                for (int i = t; i < m; i += NT)
                    reinterpret_cast<d2*>(a.optY)[(long long)(j0 + r) * m + i] =
                        reinterpret_cast<const d2*>(a.Yn)[(long long)(j0 + r) * m + i];
    // T = (Y - M/mu) - A V.  A block with a realisation whose V is not the previous X runs the
    // digit-plane product (apply_A's block body, digit stages in the Ad region, T into Ts; the
    // realisations with RealState::avok take A V = AX there too); otherwise T is formed here as
    // (Y - M/mu) - AX with the same expression.
    int need = 0;
    if (a.LA && t < GRB) need = live_s[t] && !avok_s[t];
    if (__syncthreads_or(need)) {
        for (int idx = t; idx < GRB * tst; idx += NT) Ts[idx] = make_double2(0.0, 0.0);   // padding, dead rows
        __syncthreads();
        i8a_block<true>(nb, a.n, m, i8_nks_dev(a.n), reinterpret_cast<const i4v*>(a.LA), a.Z, a.N, a.Yo, a.M,
                        reinterpret_cast<double*>(Ts), 2 * tst, a.c8, a.rs, a.zeros, a.AX,
                        reinterpret_cast<int8_t(*)[ROWS * RSA]>(Ad), sc_s, p2_s, live_s, avok_s, j0, 0);
    } else if (early) {
        // T formed from the early loads above
    } else
    for (int idx = t; idx < GRB * mp; idx += NT) {
        const int jl = idx / mp, k = idx - jl * mp, j = j0 + jl;
        d2 v = make_double2(0.0, 0.0);
        if (live_s[jl] && k < m) {
            const long long o = (long long)j * m + k;
            if (avok_s[jl]) {
                const d2 y = reinterpret_cast<const d2*>(a.Yo)[o], mm = reinterpret_cast<const d2*>(a.M)[o],
                         ax = reinterpret_cast<const d2*>(a.AX)[o];
                const double im = imu0_s[jl];
                v = make_double2(fma(-mm.x, im, y.x) - ax.x, fma(-mm.y, im, y.y) - ax.y);
            } else {
                v = reinterpret_cast<const d2*>(a.T)[o];
            }
        }
        Ts[jl * tst + k] = v;
    }
    __syncthreads();
    STAMP(1);

    // ---- g = G T: wave w owns output tiles 2w, 2w + 1 (16 complex each)
    const int nct = mp / 16, nks = mp / 4, nstage = nks / GSK;
    const int ct0 = min(2 * w, nct - 1), ct1 = min(2 * w + 1, nct - 1);
    const d2* gp0 = reinterpret_cast<const d2*>(a.Gf) + (long long)ct0 * 64 + lane;
    const d2* gp1 = reinterpret_cast<const d2*>(a.Gf) + (long long)ct1 * 64 + lane;
    auto gload = [&](GSet& gs, int s) {
#pragma unroll
        for (int kk = 0; kk < GSK; ++kk) {
            const long long ks = min(GSK * s + kk, nks - 1);
#ifdef ACE_GYK_PROBE_NO_G
            gs.f[kk][0] = make_double2(1.0 + ks, 0.5);
            gs.f[kk][1] = make_double2(0.5, 1.0 + ks);
#else
            gs.f[kk][0] = gp0[ks * nct * 64];
            gs.f[kk][1] = gp1[ks * nct * 64];
#endif
        }
    };
    d4v p1[2], p2[2], p3[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) p1[c] = p2[c] = p3[c] = d4v{0.0, 0.0, 0.0, 0.0};
    const d2* trow = Ts + (lane & 15) * tst + (lane >> 4);
    struct TSet {
        d2 v[GSK];
    };
    auto tload = [&](TSet& ts, int s) {   // T fragments of a stage, one stage ahead of their use
        const int s2 = min(s, nstage - 1);
#pragma unroll
        for (int kk = 0; kk < GSK; ++kk) ts.v[kk] = trow[4 * (GSK * s2 + kk)];
    };
    auto gcomp = [&](const GSet& gs, const TSet& ts) {
#pragma unroll
        for (int kk = 0; kk < GSK; ++kk) {
            const d2 v = ts.v[kk];
            const double ar = v.x, ai = v.y, as = v.x + v.y;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const d2 l = gs.f[kk][c];
                p1[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar, l.x, p1[c], 0, 0, 0);
                p2[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai, l.y, p2[c], 0, 0, 0);
                p3[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(as, l.x + l.y, p3[c], 0, 0, 0);
            }
        }
    };
    {
        GSet gA, gB;
        TSet tA, tB;
        gload(gA, 0);
        tload(tA, 0);
        for (int s = 0; s < nstage; s += 2) {   // nstage is even (mp multiple of 32)
            gload(gB, s + 1);
            tload(tB, s + 1);
            __builtin_amdgcn_sched_barrier(0);
            gcomp(gA, tA);
            __builtin_amdgcn_sched_barrier(0);
            gload(gA, s + 2);
            tload(tA, s + 2);
            __builtin_amdgcn_sched_barrier(0);
            gcomp(gB, tB);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // the Y-step inputs of the lane's 8 elements as one batch of loads (unconditional, clamped
    // addresses; per-element branches would serialise 8 memory round trips).  Issued after the
    // G T loop: held across it they would push the kernel past 256 VGPRs into scratch.
    d2 mi[2][4], yov[2][4], sov[2][4];
    double biv[2][4], muv[4];
    const bool mspl = GLDS && a.msp;   // (m-space: S of the lane's outputs in the same batch)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int jl = (lane >> 4) + 4 * r;
        muv[r] = mu_s[jl];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int i = min(16 * (2 * w + c) + (lane & 15), m - 1);
            const long long off = (long long)(live_s[jl] ? j0 + jl : j0) * m + i;
            mi[c][r] = reinterpret_cast<const d2*>(a.M)[off];
            yov[c][r] = reinterpret_cast<const d2*>(a.Yo)[off];
            biv[c][r] = a.B[off];
            sov[c][r] = mspl ? reinterpret_cast<const d2*>(a.Sold)[off] : make_double2(0.0, 0.0);
        }
    }
    __syncthreads();   // every wave is done with T: Ts becomes Y_new
    STAMP(2);
#ifdef ACE_GYK_PROBE_ONLY_A
    {
        double sacc = 0.0;
        for (int c = 0; c < 2; ++c)
            for (int r = 0; r < 4; ++r) sacc += p1[c][r] + p2[c][r] + p3[c][r];
        if (sacc == 12345.678) a.g[0] = sacc;
    }
    return;
#endif

    // ---- Y-step on this lane's 2 x 4 outputs: realisation (lane >> 4) + 4 r, output 16 ct + (lane & 15)
    double v7[4][9];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < 9; ++k) v7[r][k] = 0.0;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int ct = 2 * w + c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int jl = (lane >> 4) + 4 * r, j = j0 + jl, i = 16 * ct + (lane & 15);
            if (ct >= nct || i >= m || !live_s[jl]) continue;
            const long long off = (long long)j * m + i;
            const double mu = muv[r];
            const d2 mii = mi[c][r], yo = yov[c][r];
            d2 gv, ax, mn, y;
            ystep_elem(p1[c][r], p2[c][r], p3[c][r], mu, mii, yo, biv[c][r], gv, ax, mn, y, v7[r]);
            if constexpr (!GLDS) reinterpret_cast<d2*>(a.g)[off] = gv;
            if (a.AX) reinterpret_cast<d2*>(a.AX)[off] = ax;
            reinterpret_cast<d2*>(a.M)[off] = mn;
            reinterpret_cast<d2*>(a.Yn)[off] = y;
            if constexpr (GLDS) {
                if (msp_s[jl]) {   // m-space candidate: Re (A Z)^H g, g^H K g = Re g^H (T - g), S' = S + g
                    msp_sums_elem(yo, mii, 1.0 / mu, Ts[jl * tst + i], gv, v7[r]);
                    const d2 so = ent_s[jl] ? make_double2(0.0, 0.0) : sov[c][r];
                    d2* sn = reinterpret_cast<d2*>(a.Snew) + off;
                    // deferred opt_S (RealState::optsrc 4 / 5): the best iterate's S is the one this
                    // store overwrites -- keep it first (rare: no better iterate for two iterations)
                    if (oss_s[jl] == 4 + (a.it & 1)) reinterpret_cast<d2*>(a.optS)[off] = *sn;
                    *sn = cadd(so, gv);
                }
                Ts[jl * tst + i] = gv;   // g stays on chip for the fused apply_AH
            } else {
                Ts[jl * tst + i] = y;
            }
        }
    }
#ifdef ACE_GYK_PROBE_P1
    return;
#endif
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int k = 0; k < 5; ++k) v7[r][k] = bsum16(v7[r][k]);
        v7[r][5] = bmax16(v7[r][5]);
        v7[r][6] = bsum16(v7[r][6]);
        if (GLDS && a.msp) {
            v7[r][7] = bsum16(v7[r][7]);
            v7[r][8] = bsum16(v7[r][8]);
        }
        if ((lane & 15) == 0)
#pragma unroll
            for (int k = 0; k < 9; ++k) red[w][(lane >> 4) + 4 * r][k] = v7[r][k];
    }
    __syncthreads();
    STAMP(3);
    if (t < GRB) {
        double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int q = 0; q < 8; ++q) {   // fixed order over the waves
#pragma unroll
            for (int k = 0; k < 5; ++k) v[k] += red[q][t][k];
            v[5] = fmax(v[5], red[q][t][5]);
            v[6] += red[q][t][6];
            v[7] += red[q][t][7];
            v[8] += red[q][t][8];
        }
        int imp = 0;
        double p2 = 1.0, sc = 0.0;
        if (live_s[t]) {
            RealState& rs = a.rs[j0 + t];
            rs.obj2 = v[0];
            rs.nAX2 = v[1];
            rs.nY2 = v[2];
            rs.nJM2 = v[3];
            rs.dY2 = v[4];
            imp = sqrt(v[0]) < rs.opt_obj;   // iter_control makes the same decision (opt_Y here)
            plane_scale(v[5] + v[6], a.c8[1], p2, sc);
            if (a.yn_id)   // opt_Y deferred: Y_new stays in Yn until that buffer comes round again
                rs.optysrc = imp ? a.yn_id : (oys_s[t] == a.yn_id ? 0 : oys_s[t]);
            if (msp_s[t]) {   // the fused pass's sums, from m-space (RealState::msp)
                const double s0 = rs.fs0 + 2.0 * v[7] + v[8];   // ||Z + A^H g||^2
                const double s3 = v[8];                         // ||A^H g||^2
                bool take = !ent_s[t];
                if (!take) {   // entry: the bound of fused_control with `room` more steps like this one
                    const bool r1 = a.rank_one && a.rank_one[j0 + t];
                    const int np = r1 ? 1 : a.np;
                    const double cum = rs.kfcum + a.room * sqrt(s3);
                    take = s0 > 0.0;
                    for (int p = 0; p < 4 && p < np; ++p) {
                        const double fl = r1 ? 0.95 : a.fl[p], lb = rs.kf[p] * (1.0 - 1e-12) - cum;
                        take = take && lb > 0.0 && lb * lb > fl * s0 * (1.0 + 1e-9);
                    }
                }
                if (take) {
                    atomicAdd(a.dc.done_count + 1, 1);   // m-space step count (ace_prof_msp_steps)
                    rs.fs0 = s0;
                    rs.fs3 = s3;
                    rs.fzit = a.it;
                    rs.mzit = a.it;
                    if (ent_s[t]) {
                        rs.msp = 1;
                        rs.z0id = (a.it & 1) ? 1 : 2;   // the Z buffer this iteration reads (Zc)
                        rs.msp_pad = a.it;               // (entry iteration: no S before it)
                    }
                }
                if (oss_s[t] == 4 + (a.it & 1)) rs.optsrc = 3;   // (saved to opt_S in the loop above)
                // the Z-step's certificate and control right here, on the state in place (the
                // Z-step launch then returns at once for this realisation, RealState::zit); not at
                // the last iteration, whose pending tests need the one-wave dual_fixup
                if constexpr (GLDS) {
                    if (take && za_ctl && !za.fixup_now) fused_control<false>(za, &rs, z_profile(za, j0 + t));
                }
                msp_s[t] = take;
            }
        }
        imp_s[t] = imp;
        p2_s[t] = p2;
        sc_s[t] = sc;
    }
    __syncthreads();
    STAMP(4);
#ifdef ACE_GYK_PROBE_P2
    return;
#endif
    for (int idx = t; idx < GRB * m; idx += NT) {   // opt_Y (:344-351)
        const int jl = idx / m, i = idx - jl * m;
        if (!a.yn_id && live_s[jl] && imp_s[jl])
            reinterpret_cast<d2*>(a.optY)[(long long)(j0 + jl) * m + i] = Ts[jl * tst + i];
    }
    if (a.lazy) {   // no K Y: the Z-step forms the dual terms when the test needs them
        STAMP(5);
        STAMP_PRINT("gyk-lazy T|GT|Ystep+shfl|red+RS|optY:", 6);
        return;
    }
#ifdef ACE_GYK_PROBE_P3
    return;
#endif
    // ---- K Y_new: digit planes of Y_new (thread: realisation bl, entries 64 s + 2 cp + {0, 1})
    {
        const int bl = t >> 5, cp = t & 31;
        const double p2 = p2_s[bl];
        for (int s = 0; s < nksK / KSC; ++s) {
            d2 x[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int k = 64 * s + 2 * cp + u;
                x[u] = (live_s[bl] && k < m) ? Ts[bl * tst + k] : make_double2(0.0, 0.0);
            }
            const double v[4] = {x[0].x, x[0].y, x[1].x, x[1].y};
            uint32_t d[8];
            digits4(v, p2, d);
#pragma unroll
            for (int tt = 0; tt < 8; ++tt) *reinterpret_cast<uint32_t*>(&Ad[lds_row(bl, tt) * rst + KC * s + 4 * cp]) = d[tt];
        }
    }
    __syncthreads();
    STAMP(5);
#ifdef ACE_GYK_PROBE_NO_C
    return;
#endif
    const int h = lane >> 5, ldo = 2 * m, ocb = NCB / 2, ncb = (ldo + ocb - 1) / ocb;
    const int8_t* arow = &Ad[(lane & 31) * rst + 16 * (lane >> 5)];
    const i4v* Bf = reinterpret_cast<const i4v*>(a.LK);
    const int total = ncb * nksK;
    auto bfl = [&](BSet& b, int f0) {
#pragma unroll
        for (int kk = 0; kk < SK; ++kk) {
            const int f = min(f0 + kk, total - 1), cb = f / nksK, ks = f - cb * nksK;
            const i4v* pp = Bf + ((long long)(cb * (NCB / 32) + 2 * w) * nksK + ks) * 64 + lane;
            b.f[kk][0] = pp[0];
            b.f[kk][1] = pp[(long long)nksK * 64];
        }
    };
    const double* Ysd = reinterpret_cast<const double*>(Ts);
    double dacc[4][2], nacc[4][2];
#pragma unroll
    for (int R = 0; R < 4; ++R) dacc[R][0] = dacc[R][1] = nacc[R][0] = nacc[R][1] = 0.0;
    auto epilogue = [&](int cbk, i16v (&acc)[4][2]) {
        const int col = (cbk * (NCB / 64) + w) * 32 + (lane & 31), colc = min(col, ldo - 1);
        double yo[4][2], ko[4][2];   // Y0, KY0 of the lane's 8 outputs, loaded as one batch
#pragma unroll
        for (int R = 0; R < 4; ++R)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int blo = 4 * R + 2 * q + h;
                const long long off = (long long)(live_s[blo] ? j0 + blo : j0) * ldo + colc;
                yo[R][q] = a.Yo[off];
                ko[R][q] = a.KYo[off];
            }
#pragma unroll
        for (int R = 0; R < 4; ++R)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int blo = 4 * R + 2 * q + h, j = j0 + blo;
                if (!live_s[blo] || col >= ldo) continue;
                i16v cmb;
#pragma unroll
                for (int e = 0; e < 16; ++e) cmb[e] = acc[R][0][e] + 128 * acc[R][1][e];
                const double kyn = sc_s[blo] * recombine(cmb, q);
                const long long off = (long long)j * ldo + col;
                a.KYn[off] = kyn;
                const double yn = Ysd[2 * blo * tst + col];
                dacc[R][q] += (yn - yo[R][q]) * (kyn - ko[R][q]);
                nacc[R][q] += yn * kyn;
            }
#pragma unroll
        for (int R = 0; R < 4; ++R) acc[R][0] = acc[R][1] = i16v{};
    };
    i16v acc[4][2];
#pragma unroll
    for (int R = 0; R < 4; ++R) acc[R][0] = acc[R][1] = i16v{};
    BSet bA, bB;
    bfl(bA, 0);
    for (int f = 0; f < total; f += 2 * SK) {
        bfl(bB, f + SK);
        __builtin_amdgcn_sched_barrier(0);
        stage_mma(arow + 32 * (f % nksK), rst, bA, acc);
        __builtin_amdgcn_sched_barrier(0);
        bfl(bA, f + 2 * SK);
        __builtin_amdgcn_sched_barrier(0);
        stage_mma(arow + 32 * ((f + SK) % nksK), rst, bB, acc);
        __builtin_amdgcn_sched_barrier(0);
        if ((f + 2 * SK) % nksK == 0) epilogue(f / nksK, acc);
    }
    STAMP(6);
    // dual terms: lanes of one half-wave share realisations; then the 8 waves in fixed order
#pragma unroll
    for (int R = 0; R < 4; ++R)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) {
                dacc[R][q] += __shfl_xor(dacc[R][q], o, 64);
                nacc[R][q] += __shfl_xor(nacc[R][q], o, 64);
            }
            if ((lane & 31) == 0) {
                red[w][4 * R + 2 * q + h][0] = dacc[R][q];
                red[w][4 * R + 2 * q + h][1] = nacc[R][q];
            }
        }
    __syncthreads();
    if (t < GRB && live_s[t]) {
        double dv = 0.0, nv = 0.0;
        for (int q = 0; q < 8; ++q) {
            dv += red[q][t][0];
            nv += red[q][t][1];
        }
        a.rs[j0 + t].dAtY = dv;
        a.rs[j0 + t].nAtY = nv;
    }
    STAMP(7);
    STAMP_PRINT("gyk T|GT|Ystep+shfl|red+RS|optY+digits|KY|dual:", 8);
}
__global__ __launch_bounds__(NT, 1) void gyk_kernel(int nb, int m, GykArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    gyk_body<false>(nb, m, a, smem, ZArgs{}, 0);
}
// One iteration's matrix work in one launch (unit path, lazy dual residual, fused Z-step pass):
// gyk_body (T, g = G T, the Y-step; g left in the LDS rows of T), then the fused apply_AH body
// on the same 16 realisations with its digit planes staged from LDS.  The g round trip through
// HBM, apply_AH's g loads and one launch boundary go away.  LDS: [T / g rows | digit planes]
// and the 64 KiB of Z-step partial sums over the T rows when they are large enough, else after.
__host__ __device__ __forceinline__ size_t gyf_ts_bytes(int m) { return ((size_t)GRB * (gyk_mp(m) + 1) * 16 + 255) & ~(size_t)255; }
__global__ __launch_bounds__(NT, 1) void gyf_kernel(int nb, int m, int n, GykArgs a, const i4v* __restrict__ LAH,
                                                    double* __restrict__ Wp, ZArgs za, size_t ad_bytes, int za_ctl) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // msr_kernel already ran this iteration (and possibly later ones) for every live realisation
    // of the block (RealState::mzit >= it): nothing to do (never the case in the regular flow)
    {
        const int j = blockIdx.x * GRB + (int)threadIdx.x;
        const bool behind = threadIdx.x < GRB && j < nb && !a.rs[j].done && a.rs[j].mzit < a.it;
        if (!__syncthreads_or(behind)) return;
    }
    gyk_body<true>(nb, m, a, smem, za, za_ctl);
    __syncthreads();
    const size_t ts = gyf_ts_bytes(m);
    int8_t* Ad = reinterpret_cast<int8_t*>(smem + ts);
    double* zsum = reinterpret_cast<double*>(ts >= (size_t)8 * 8 * 2 * 64 * sizeof(double) ? smem : smem + ts + ad_bytes);
    i8ah_body<false, true, true>(nb, m, n, i8_nks_dev(m), LAH, nullptr, Wp, a.c8, a.rs, za, Ad, zsum,
                                 reinterpret_cast<const d2*>(smem), gyk_mp(m) + 1);
}

// ---- m-space run (msr_kernel): the m-space steady state of gyf_kernel (RealState::msp) iterated
// inside one launch.  Once every live realisation of a 16-realisation block is in the m-space form,
// an iteration is T = (Y - M/mu) - AX, g = G T, the Y-step, S' = S + g and the certified control
// (fused_control): no n-vector, no Z-step, and nothing of one realisation that another needs.  The
// work-group keeps Y, M, AX and B of its 16 realisations in registers and S in LDS across
// iterations, so an iteration moves no per-realisation state through HBM (only G, from L2), and there
// is no launch boundary between iterations.  The arithmetic is gyf_kernel's (same T expression, the
// same MFMA sequence for g, ystep_elem / msp_sums_elem, the same reduction order, fused_control), so
// the iterates are bit-identical to the per-iteration launches.  The run stops at it_end, or after
// the iteration in which some realisation's bound fails (its Z-step must run: resume = it) or its
// convergence test is left pending (the next gyf_kernel finishes it: resume = it + 1); it then writes
// the state back where the per-iteration launches expect it, and *resume gets the smallest
// iteration the regular launches must run from.  A block that is not entirely in the m-space form
// at it0 returns at once (resume = it0).  Stopped realisations (convergence mode) write their state
// back at the stop and drop out.
constexpr int MGSK = 2;   // G T pipeline depth here (registers hold the state; the k order is gyk_body's)
__host__ __device__ __forceinline__ size_t msr_lds_bytes() { return (size_t)GRB * 257 * 16 + (size_t)4096 * 16; }
// TPW output tiles of 16 per wave: 2 (8 waves of 256 VGPRs) or 4 (4 waves, one per SIMD, with the
// whole register file); the per-realisation sums keep the 8-wave partial order (red[8]) either way
template <int TPW>
__global__ __launch_bounds__(64 * 16 / TPW, 1) void msr_kernel(MsrArgs a, ZArgs za) {
    constexpr int NTW = 64 * 16 / TPW;   // threads
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int mp = 256, tst = mp + 1, nct = mp / 16, nks = mp / 4, nstage = nks / MGSK;
    d2* Ts = reinterpret_cast<d2*>(smem);        // [16][tst]: T
    d2* Ss = Ts + GRB * tst;                     // [4 TPW][NTW]: S of the thread's outputs (thread-private)
    __shared__ double red[8][GRB][9];
    __shared__ double mu_s[GRB];
    __shared__ int live_s[GRB], flg_s[GRB];
    __shared__ RealState rsl[GRB];   // the block's control blocks for the run (written back at its end)
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, j0 = blockIdx.x * GRB, m = a.m;
    int bad = 0, ahead = 0, res = 0x7fffffff;
    if (t < GRB) {
        const int j = j0 + t;
        const bool lv = j < a.nb && !a.rs[j].done;
        live_s[t] = lv;
        mu_s[t] = lv ? a.rs[j].mu : 1.0;
        int fl = 0;
        if (lv) {
            RealState& r = a.rs[j];
            ahead = r.mzit >= a.it0;   // an earlier run took the block past it0: its resume point stands
            res = r.mres;
            bad = !r.msp || r.dpend || r.mzit != a.it0 - 1 || r.zit != a.it0 - 1;
            // deferred best iterates (opt_Y in a Y buffer, opt_S in an S buffer) go to opt_Y / opt_S
            // now: the run keeps Y and S on chip and writes an improved iterate straight there
            if (!bad) {
                if (r.optysrc == 1 || r.optysrc == 2) fl |= r.optysrc;
                if (r.optsrc == 4 || r.optsrc == 5) fl |= (r.optsrc - 3) << 2;
            }
        }
        flg_s[t] = fl;
    }
    if (__syncthreads_or(ahead)) {
        if (t < GRB && ahead) atomicMin(a.resume, res);
        return;
    }
    if (__syncthreads_or(bad)) {
        if (t == 0) {
            atomicMin(a.resume, a.it0);
            atomicAdd(a.steps + 1, 1);   // (diagnostics: blocks not ready at it0)
        }
        return;
    }
    if (!__syncthreads_or(t < GRB && live_s[t])) return;
    // the thread's outputs: realisation jl(r) = (lane >> 4) + 4 r, entry i(c) = 16 (2 w + c) + (lane & 15)
    // (the f64 MFMA accumulator map of g = G T)
    bool lv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) lv[r] = live_s[(lane >> 4) + 4 * r];
    auto off = [&](int r, int c) -> long long {
        return (long long)(lv[r] ? j0 + (lane >> 4) + 4 * r : j0) * m + 16 * (TPW * w + c) + (lane & 15);
    };
    int vw = 0;   // m-vectors realisation t writes (MsrArgs::vecw)
    if (t < GRB && live_s[t]) vw = ((flg_s[t] & 3) ? 1 : 0) + ((flg_s[t] >> 2) ? 1 : 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int fl = flg_s[(lane >> 4) + 4 * r];
        if (!lv[r] || !fl) continue;
#pragma unroll
        for (int c = 0; c < TPW; ++c) {
            if (fl & 3) reinterpret_cast<d2*>(a.optY)[off(r, c)] = reinterpret_cast<const d2*>(a.Y[(fl & 3) - 1])[off(r, c)];
            if (fl >> 2) reinterpret_cast<d2*>(a.optS)[off(r, c)] = reinterpret_cast<const d2*>(a.S[(fl >> 2) - 1])[off(r, c)];
        }
    }
    if (t < GRB && live_s[t]) {
        rsl[t] = a.rs[j0 + t];
        if (flg_s[t] & 3) rsl[t].optysrc = 0;
        if (flg_s[t] >> 2) rsl[t].optsrc = 3;
    }
    // state of iterate it0 - 1.  AX lives in the T tile between iterations: the thread's slot (jl, i) holds
    // AX from its Y-step until its T formation reads it and writes T there (registers: 32 VGPRs fewer)
    d2 yv[TPW][4], mv[TPW][4];
    double bv[TPW][4];
    {
        const int p = (a.it0 - 1) & 1;
#pragma unroll
        for (int c = 0; c < TPW; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const long long o = off(r, c);
                yv[c][r] = reinterpret_cast<const d2*>(a.Y[p])[o];
                mv[c][r] = reinterpret_cast<const d2*>(a.M)[o];
                Ts[((lane >> 4) + 4 * r) * tst + 16 * (TPW * w + c) + (lane & 15)] = reinterpret_cast<const d2*>(a.AX)[o];
                bv[c][r] = a.B[o];
                Ss[(4 * c + r) * NTW + t] = reinterpret_cast<const d2*>(a.S[p])[o];
            }
    }
    __syncthreads();   // (every thread is done with the flush flags)
    if (t < GRB) flg_s[t] = 0;
    const d2* gp = reinterpret_cast<const d2*>(a.Gf) + (long long)(TPW * w) * 64 + lane;   // tile TPW w + c: + 64 c
    const d2* trow = Ts + (lane & 15) * tst + (lane >> 4);
    int cnt = 0;   // m-space steps of realisation t (ace_prof_msp_steps)
    bool mylive = t < GRB && live_s[t] && !(flg_s[t] & 4);
    // best iterates, deferred like gyf_kernel's opt_Y / opt_S: the previous iterate's Y (in yv) and S
    // (in Ss) are written out only when the next iterate does not improve on them (or the run ends)
    bool pbY = false, pbS = false;
#ifdef ACE_MSR_STAMPS   // phase times of block 5, summed over its iterations (10 ns units)
    unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tp = __builtin_amdgcn_s_memrealtime();
#define MSR_STAMP(k) do { if (blockIdx.x == 5 && t == 0) { const unsigned long long tn = __builtin_amdgcn_s_memrealtime(); ph[k] += tn - tp; tp = tn; } } while (0)
#else
#define MSR_STAMP(k)
#endif
    for (int it = a.it0;; ++it) {
        // T = (Y - M/mu) - AX (gyk_body's t_from expression)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int jl = (lane >> 4) + 4 * r;
            const double im = lv[r] ? 1.0 / mu_s[jl] : 0.0;
#pragma unroll
            for (int c = 0; c < TPW; ++c) {
                d2* slot = &Ts[jl * tst + 16 * (TPW * w + c) + (lane & 15)];
                d2 v = make_double2(0.0, 0.0);
                if (lv[r]) {
                    const d2 xv = *slot;   // AX of the previous Y-step
                    v = make_double2(fma(-mv[c][r].x, im, yv[c][r].x) - xv.x, fma(-mv[c][r].y, im, yv[c][r].y) - xv.y);
                }
                *slot = v;
            }
        }
        __syncthreads();
        MSR_STAMP(0);
        // g = G T: gyk_body's 3M product, the same k order
        d4v p1[TPW], p2[TPW], p3[TPW];
#pragma unroll
        for (int c = 0; c < TPW; ++c) p1[c] = p2[c] = p3[c] = d4v{0.0, 0.0, 0.0, 0.0};
        {
            struct GS {
                d2 f[MGSK][TPW];
            };
            struct TS {
                d2 v[MGSK];
            };
            auto gload = [&](GS& gs, int s) {
#pragma unroll
                for (int kk = 0; kk < MGSK; ++kk) {
                    const long long ks = min(MGSK * s + kk, nks - 1);
#pragma unroll
                    for (int c = 0; c < TPW; ++c) gs.f[kk][c] = gp[ks * nct * 64 + 64 * c];
                }
            };
            auto tload = [&](TS& ts, int s) {
                const int s2 = min(s, nstage - 1);
#pragma unroll
                for (int kk = 0; kk < MGSK; ++kk) ts.v[kk] = trow[4 * (MGSK * s2 + kk)];
            };
            auto gcomp = [&](const GS& gs, const TS& ts) {
#pragma unroll
                for (int kk = 0; kk < MGSK; ++kk) {
                    const d2 v = ts.v[kk];
                    const double ar = v.x, ai = v.y, as = v.x + v.y;
#pragma unroll
                    for (int c = 0; c < TPW; ++c) {
                        const d2 l = gs.f[kk][c];
                        p1[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar, l.x, p1[c], 0, 0, 0);
                        p2[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai, l.y, p2[c], 0, 0, 0);
                        p3[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(as, l.x + l.y, p3[c], 0, 0, 0);
                    }
                }
            };
            GS gA, gB;
            TS tA, tB;
            gload(gA, 0);
            tload(tA, 0);
            for (int s = 0; s < nstage; s += 2) {
                gload(gB, s + 1);
                tload(tB, s + 1);
                __builtin_amdgcn_sched_barrier(0);
                gcomp(gA, tA);
                __builtin_amdgcn_sched_barrier(0);
                gload(gA, s + 2);
                tload(tA, s + 2);
                __builtin_amdgcn_sched_barrier(0);
                gcomp(gB, tB);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        MSR_STAMP(1);
        __syncthreads();   // every wave has read T: the Y-step writes AX into its slots
        MSR_STAMP(2);
        // Y-step and m-space sums.  gyk_body runs c outer, r inner; each sum v7[r][k] still adds its
        // c = 0 term first, so r outer (one r's sums live at a time) rounds identically.
        d2 yn[TPW][4], sn[TPW][4];   // Y' and S' (S of the previous iterate stays in Ss until the control)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int jl = (lane >> 4) + 4 * r;
#pragma unroll
          for (int h = 0; h < TPW / 2; ++h) {   // tile pair h: the sums of 8-wave wave TPW w / 2 + h
            double v7[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) v7[k] = 0.0;
#pragma unroll
            for (int c = 2 * h; c < 2 * h + 2; ++c) {
                const int i = 16 * (TPW * w + c) + (lane & 15);
                yn[c][r] = sn[c][r] = make_double2(0.0, 0.0);
                if (!lv[r]) continue;
                const double mu = mu_s[jl];
                d2 gv, ax, mn, y;
                ystep_elem(p1[c][r], p2[c][r], p3[c][r], mu, mv[c][r], yv[c][r], bv[c][r], gv, ax, mn, y, v7);
                msp_sums_elem(yv[c][r], mv[c][r], 1.0 / mu, Ts[jl * tst + i], gv, v7);
                sn[c][r] = cadd(Ss[(4 * c + r) * NTW + t], gv);
                yn[c][r] = y;
                mv[c][r] = mn;
                Ts[jl * tst + i] = ax;
            }
#pragma unroll
            for (int k = 0; k < 5; ++k) v7[k] = bsum16(v7[k]);
            v7[5] = bmax16(v7[5]);
            v7[6] = bsum16(v7[6]);
            v7[7] = bsum16(v7[7]);
            v7[8] = bsum16(v7[8]);
            if ((lane & 15) == 0)
#pragma unroll
                for (int k = 0; k < 9; ++k) red[TPW / 2 * w + h][jl][k] = v7[k];
          }
        }
        __syncthreads();
        MSR_STAMP(3);
        // the control of realisation t (gyk_body's m-space branch, then fused_control in place)
        if (t < GRB) {
            int fl = 0;
            if (mylive) {
                double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                for (int q = 0; q < 8; ++q) {   // fixed order over the waves
#pragma unroll
                    for (int k = 0; k < 5; ++k) v[k] += red[q][t][k];
                    v[5] = fmax(v[5], red[q][t][5]);
                    v[6] += red[q][t][6];
                    v[7] += red[q][t][7];
                    v[8] += red[q][t][8];
                }
                RealState& rs = rsl[t];
                rs.obj2 = v[0];
                rs.nAX2 = v[1];
                rs.nY2 = v[2];
                rs.nJM2 = v[3];
                rs.dY2 = v[4];
                const bool imp = sqrt(v[0]) < rs.opt_obj;
                rs.fs0 = rs.fs0 + 2.0 * v[7] + v[8];
                rs.fs3 = v[8];
                rs.fzit = it;
                rs.mzit = it;
                ++cnt;
                const int ok = fused_control<false>(za, &rs, z_profile(za, j0 + t), it);
                // opt_Y follows every improvement; opt_S an improvement whose bound held (after a failed
                // one the Z-step records X itself).  A pending best that this iterate does not beat is
                // written now (bits 1, 2); the new pending ones are written if the run ends here (64, 128)
                if (pbY && !imp) fl |= 1;
                if (pbS && !imp) fl |= 2;
                pbY = imp;
                pbS = imp && (ok & 1);
                if (pbY) fl |= 64;
                if (pbS) {
                    fl |= 128;
                    rs.optsrc = 3;                       // (fused_control's deferral, resolved here)
                }
                if (!(ok & 1)) fl |= 8;                  // the bound failed: the Z-step of `it` runs
                if (ok & 2) fl |= 16;                    // convergence test pending: the next gyf_kernel finishes it
                fl |= rs.done ? 4 : 32;                  // stopped (convergence mode) / still live
                mylive = !rs.done;
                mu_s[t] = rs.mu;
            }
            flg_s[t] = fl;
        }
        __syncthreads();
        MSR_STAMP(4);
        int any = 0;
#pragma unroll
        for (int q = 0; q < GRB; ++q) {
            const int f = flg_s[q];
            any |= f;
        }
        const bool alive = any & 32;
        const bool stop = (any & 24) || it + 1 >= a.it_end || !alive;
        if (t < GRB) {
            const int f = flg_s[t];
            vw += (f & 1) + ((f >> 1) & 1);
            if (f & (4 | 32) && (stop || (f & 4))) vw += 6 + ((f >> 6) & 1) + ((f >> 7) & 1);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (!lv[r]) continue;
            const int f = flg_s[(lane >> 4) + 4 * r];
            const bool wb = stop || (f & 4);   // leave the state where the per-iteration launches read it
            const int jl = (lane >> 4) + 4 * r;
#pragma unroll
            for (int c = 0; c < TPW; ++c) {
                const int i = 16 * (TPW * w + c) + (lane & 15);
                const long long o = (long long)(j0 + jl) * m + i;
                d2* ssl = &Ss[(4 * c + r) * NTW + t];
                if (f & 1) reinterpret_cast<d2*>(a.optY)[o] = yv[c][r];   // the previous iterate's
                if (f & 2) reinterpret_cast<d2*>(a.optS)[o] = *ssl;
                if (wb && (f & 64)) reinterpret_cast<d2*>(a.optY)[o] = yn[c][r];
                if (wb && (f & 128)) reinterpret_cast<d2*>(a.optS)[o] = sn[c][r];
                if (wb) {
                    reinterpret_cast<d2*>(a.Y[it & 1])[o] = yn[c][r];
                    reinterpret_cast<d2*>(a.Y[(it + 1) & 1])[o] = yv[c][r];
                    reinterpret_cast<d2*>(a.M)[o] = mv[c][r];
                    reinterpret_cast<d2*>(a.AX)[o] = Ts[jl * tst + i];
                    reinterpret_cast<d2*>(a.S[it & 1])[o] = sn[c][r];
                    reinterpret_cast<d2*>(a.S[(it + 1) & 1])[o] = *ssl;
                }
                *ssl = sn[c][r];
                yv[c][r] = yn[c][r];
            }
            if (f & 4) lv[r] = false;
        }
        MSR_STAMP(5);
        if (stop) {
#ifdef ACE_MSR_STAMPS
            if (blockIdx.x == 5 && t == 0)
                printf("msr it %d..%d: T %llu GT %llu bar %llu Ystep %llu ctl %llu wb %llu (x10ns)\n", a.it0, it,
                       ph[0], ph[1], ph[2], ph[3], ph[4], ph[5]);
#endif
            const int rp = (any & 8) ? it : it + 1;
            if (t < GRB && cnt) {
                atomicAdd(a.mspcount, cnt);
                atomicAdd(a.steps, cnt);
            }
            if (t < GRB && vw && a.vecw) atomicAdd(a.vecw, vw);
            if (t < GRB && live_s[t]) {   // (stopped realisations were written back at their stop)
                if (mylive) rsl[t].mres = rp;
                a.rs[j0 + t] = rsl[t];
            }
            if (t == 0 && alive) atomicMin(a.resume, rp);
            if (t == 0 && (any & 24)) atomicAdd(a.steps + ((any & 8) ? 2 : 3), 1);   // (diagnostics)
            return;
        }
    }
}

// G [m][m] c128 -> f64 MFMA B-operand fragments: ((ks * (mp/16) + ct) * 64 + lane) holds
// G[16 ct + (lane & 15)][4 ks + (lane >> 4)] (zero padded to mp = m rounded up to 32).
__global__ __launch_bounds__(256) void gyk_gfrag_kernel(int m, const double* __restrict__ Gp, double* __restrict__ Gf) {
    const int mp = gyk_mp(m), nct = mp / 16;
    const long long e = blockIdx.x * 256LL + threadIdx.x;
    if (e >= (long long)mp * mp) return;
    const int lane = (int)(e & 63);
    const long long q = e >> 6;
    const int ct = (int)(q % nct), ks = (int)(q / nct);
    const int i = 16 * ct + (lane & 15), k = 4 * ks + (lane >> 4);
    const d2 v = (i < m && k < m) ? reinterpret_cast<const d2*>(Gp)[(long long)i * m + k] : make_double2(0.0, 0.0);
    reinterpret_cast<d2*>(Gf)[e] = v;
}

// K_int = rint(K / c^2) (exact: K = A A^H of a phase code is c^2 times a Gaussian-integer
// matrix, and its f64 rounding error is far below c^2 / 2).  Real expansion entry (oc, kk)
// of K_int as base-128 digits lo in [0, 127], hi = floor(v / 128); plane p of output tile
// oc / 32 is codebook tile 2 (oc / 32) + p.
__global__ __launch_bounds__(256) void i8k_expand_kernel(int m, const double* __restrict__ Kp,
                                                          const double* __restrict__ cmax, int8_t* __restrict__ LK,
                                                          int nks, int* flag) {
    const long long e = blockIdx.x * 256LL + threadIdx.x;
    if (e >= (long long)m * m) return;
    const int i = (int)(e / m), k = (int)(e % m);
    const d2 kv = reinterpret_cast<const d2*>(Kp)[e];
    const double c2 = cmax[1];
    const double kr = rint(kv.x / c2), ki = rint(kv.y / c2);
    if (fabs(kr) > 8192.0 || fabs(ki) > 8192.0) atomicOr(flag, 2);
    auto put = [&](int oc, int kk, double v) {
        const int iv = (int)v, hi = iv >> 7, lo = iv & 127;   // iv = 128 hi + lo
        const int t = oc >> 5, cc = oc & 31;
        LK[frag_off(32 * (2 * t) + cc, kk, nks)] = (int8_t)lo;
        LK[frag_off(32 * (2 * t + 1) + cc, kk, nks)] = (int8_t)hi;
    };
    put(2 * i, 2 * k, kr);
    put(2 * i, 2 * k + 1, -ki);
    put(2 * i + 1, 2 * k, ki);
    put(2 * i + 1, 2 * k + 1, kr);
}
}  // namespace
size_t msr_request_bytes() { return msr_lds_bytes(); }

// padded K-steps (of 32 reals) for a complex inner dimension kc: multiple of one stage
int i8_nks(int kc) { return (2 * kc + KC - 1) / KC * KSC; }
// padded 32-column tiles for mc complex outputs: multiple of one work-group's 512 columns
int i8_ncols(int mc) { return (2 * mc + NCB - 1) / NCB * NCB; }
size_t i8_frag_bytes(int mc, int kc) { return (size_t)i8_ncols(mc) * i8_nks(kc) * 32; }

void launch_i8_expand(int m, int n, const double* A, const double* cmax, int8_t* LA, int8_t* LH, int* flag,
                      hipStream_t st) {
    const long long tot = (long long)m * n;
    hipLaunchKernelGGL(i8_expand_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, m, n, A, cmax, LA,
                       i8_nks(n), LH, i8_nks(m), flag);
}

size_t i8ah_lds_bytes(int kc) { return ((size_t)ROWS * (32 * i8_nks(kc) + 16) + 255) & ~(size_t)255; }
size_t i8ah_fuse_lds_bytes() { return (size_t)8 * 8 * 2 * 64 * sizeof(double); }   // FUSE partial-sum slots

void launch_i8_apply_A(int nb, int n, int m, const int8_t* LA, const double* Z, const double* N, const double* Y,
                       const double* M, double* T, const double* cmax, const RealState* rs, const double* zeros,
                       const double* AX, hipStream_t st, int rcols) {
    dim3 grid((nb + RB - 1) / RB, i8_ncols(m) / NCB, 1), block(NT);
    hipLaunchKernelGGL(i8a_kernel, grid, block, 0, st, nb, n, m, i8_nks(n), reinterpret_cast<const i4v*>(LA), Z, N,
                       Y, M, T, cmax, rs, zeros, AX, rcols < 1 ? 1 : rcols);
}
size_t i8k_frag_bytes(int m) { return (size_t)2 * ((2 * m + NCB / 2 - 1) / (NCB / 2)) * (NCB / 2) * i8_nks(m) * 32; }
void launch_i8k_expand(int m, const double* K, const double* cmax, int8_t* LK, int* flag, hipStream_t st) {
    const long long tot = (long long)m * m;
    hipLaunchKernelGGL(i8k_expand_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, m, K, cmax, LK,
                       i8_nks(m), flag);
}
void launch_i8_apply_K(int nb, int m, const int8_t* LK, const double* Y, double* KY, const double* cmax,
                       const RealState* rs, hipStream_t st, int rcols) {
    const size_t lds = i8ah_lds_bytes(m);
    if (!lds_fits(reinterpret_cast<const void*>(&i8ah_kernel<true, false>), "i8ah_kernel<KY>", lds)) return;
    dim3 grid((nb + RB - 1) / RB, 1, 1), block(NT);
    ZArgs za{};
    za.r = rcols;
    hipLaunchKernelGGL((i8ah_kernel<true, false>), grid, block, lds, st, nb, m, m, i8_nks(m),
                       reinterpret_cast<const i4v*>(LK), Y, KY, cmax + 1, rs, za);
}
size_t gyk_gfrag_bytes(int m) { return (size_t)gyk_mp(m) * gyk_mp(m) * 16; }
size_t gyk_lds_bytes(int m) {   // Ts, then the Ad region: K Y digit planes, or apply_A's digit stages
    return (((size_t)GRB * (gyk_mp(m) + 1) * 16 + 255) & ~(size_t)255) +
           (i8ah_lds_bytes(m) > (size_t)2 * ROWS * RSA ? i8ah_lds_bytes(m) : (size_t)2 * ROWS * RSA);
}
void launch_gyk_gfrag(int m, const double* G, double* Gf, hipStream_t st) {
    const long long tot = (long long)gyk_mp(m) * gyk_mp(m);
    hipLaunchKernelGGL(gyk_gfrag_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, m, G, Gf);
}
void launch_gyk(int nb, int m, const GykArgs& a, hipStream_t st) {
    const size_t lds = gyk_lds_bytes(m);
    if (!lds_fits(reinterpret_cast<const void*>(&gyk_kernel), "gyk_kernel", lds)) return;
    hipLaunchKernelGGL(gyk_kernel, dim3((nb + GRB - 1) / GRB), dim3(NT), lds, st, nb, m, a);
}
size_t gyf_lds_bytes(int m) {
    const size_t ts = gyf_ts_bytes(m), ad = gyk_lds_bytes(m) - ts, zs = i8ah_fuse_lds_bytes();
    return ts + ad + (ts >= zs ? 0 : zs);
}
void launch_gyf(int nb, int m, int n, const GykArgs& a, const int8_t* LAH, double* W, const ZArgs& za, int ctl,
                hipStream_t st) {
    const size_t lds = gyf_lds_bytes(m);
    if (!lds_fits(reinterpret_cast<const void*>(&gyf_kernel), "gyf_kernel", lds)) return;
    const size_t ad = gyk_lds_bytes(m) - gyf_ts_bytes(m);
    hipLaunchKernelGGL(gyf_kernel, dim3((nb + GRB - 1) / GRB), dim3(NT), lds, st, nb, m, n, a,
                       reinterpret_cast<const i4v*>(LAH), W, za, ad, ctl);
}
// live realisations of [0, nb) that an m-space run starting at `it` could not take: not in the
// m-space form, a convergence test pending, or not settled through it - 1 (blocks an earlier run
// took past it count as ready)
__global__ __launch_bounds__(256) void msr_ready_kernel(int nb, const RealState* __restrict__ rs, int it, int* notready) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    int bad = 0, nm = 0, np = 0;
    if (j < nb && !rs[j].done) {
        const RealState& r = rs[j];
        bad = !r.msp || r.dpend || r.mzit < it - 1 || r.zit < it - 1;
        nm = !r.msp;
        np = r.dpend;
    }
    bad = __syncthreads_count(bad);
    nm = __syncthreads_count(nm);
    np = __syncthreads_count(np);
    if (threadIdx.x == 0 && bad) {
        atomicAdd(notready, bad);
        atomicAdd(notready + 1, nm);   // (diagnostics: not in the m-space form, test pending)
        atomicAdd(notready + 2, np);
    }
}
bool msr_supported(int m) { return m == 256; }
void launch_msr_ready(int nb, const RealState* rs, int it, int* notready, hipStream_t st) {
    hipLaunchKernelGGL(msr_ready_kernel, dim3((nb + 255) / 256), dim3(256), 0, st, nb, rs, it, notready);
}
void launch_msr(const MsrArgs& a, const ZArgs& za, int waves, hipStream_t st) {
    // waves = 4: four waves of four output tiles (one per SIMD, 256 VGPRs + 256 AGPRs) instead of
    // eight of two; measured 44 against 40 us per iteration (the 8-wave G T overlaps its waves)
    const size_t lds = msr_lds_bytes();
    if (waves == 8) {
        if (!lds_fits(reinterpret_cast<const void*>(&msr_kernel<2>), "msr_kernel<2>", lds)) return;
        hipLaunchKernelGGL(msr_kernel<2>, dim3((a.nb + GRB - 1) / GRB), dim3(512), lds, st, a, za);
    } else {
        if (!lds_fits(reinterpret_cast<const void*>(&msr_kernel<4>), "msr_kernel<4>", lds)) return;
        hipLaunchKernelGGL(msr_kernel<4>, dim3((a.nb + GRB - 1) / GRB), dim3(256), lds, st, a, za);
    }
}
// best m-space iterates still in an S ping-pong buffer (optsrc 4 / 5) -> opt_S (optsrc 3)
__global__ __launch_bounds__(256) void msp_opt_gather_kernel(int m, RealState* rs, const double* S0, const double* S1,
                                                             double* optS) {
    const int b = blockIdx.x, os = rs[b].optsrc;
    if (os != 4 && os != 5) return;
    const d2* src = reinterpret_cast<const d2*>(os == 4 ? S0 : S1) + (long long)b * m;
    d2* dst = reinterpret_cast<d2*>(optS) + (long long)b * m;
    for (int i = threadIdx.x; i < m; i += 256) dst[i] = src[i];
    if (threadIdx.x == 0) rs[b].optsrc = 3;
}
void launch_i8_msp_optx(int nb, int m, int n, const int8_t* LAH, const double* optS, double* optX, const double* cmax,
                        RealState* rs, const double* Zb1, const double* Zb2, const double* S0, const double* S1,
                        hipStream_t st) {
    hipLaunchKernelGGL(msp_opt_gather_kernel, dim3(nb), dim3(256), 0, st, m, rs, S0, S1, const_cast<double*>(optS));
    ZArgs za{};
    za.matz = 1;
    za.st = rs;
    za.Z = const_cast<double*>(Zb1);
    za.Zn = const_cast<double*>(Zb2);
    launch_i8_apply_AH(nb, m, n, LAH, optS, optX, cmax, rs, st, nullptr, &za);
}
void launch_i8_apply_AH(int nb, int m, int n, const int8_t* LAH, const double* g, double* W, const double* cmax,
                        const RealState* rs, hipStream_t st, const ZArgs* fuse, const ZArgs* plain) {
    dim3 grid((nb + RB - 1) / RB, 1, 1), block(NT);
    if (fuse) {
        const size_t lds = i8ah_lds_bytes(m) + i8ah_fuse_lds_bytes();
        if (!lds_fits(reinterpret_cast<const void*>(&i8ah_kernel<false, true>), "i8ah_kernel<FUSE>", lds)) return;
        hipLaunchKernelGGL((i8ah_kernel<false, true>), grid, block, lds, st, nb, m, n, i8_nks(m),
                           reinterpret_cast<const i4v*>(LAH), g, W, cmax, rs, *fuse);
    } else {
        const size_t lds = i8ah_lds_bytes(m);
        if (!lds_fits(reinterpret_cast<const void*>(&i8ah_kernel<false, false>), "i8ah_kernel", lds)) return;
        hipLaunchKernelGGL((i8ah_kernel<false, false>), grid, block, lds, st, nb, m, n, i8_nks(m),
                           reinterpret_cast<const i4v*>(LAH), g, W, cmax, rs, plain ? *plain : ZArgs{});
    }
}
// dynamic LDS budgets of the i8 / fused kernels (lds_dyn_budget), for the eligibility tests of ace_admm.cpp
size_t i8ah_budget(int kind) {
    const void* k = kind == 1 ? reinterpret_cast<const void*>(&i8ah_kernel<false, true>)
                  : kind == 2 ? reinterpret_cast<const void*>(&i8ah_kernel<true, false>)
                              : reinterpret_cast<const void*>(&i8ah_kernel<false, false>);
    return lds_dyn_budget(k);
}
size_t gyk_budget() { return lds_dyn_budget(reinterpret_cast<const void*>(&gyk_kernel)); }
size_t gyf_budget() { return lds_dyn_budget(reinterpret_cast<const void*>(&gyf_kernel)); }

}  // namespace ace
