// Two-stage Hermitian eigensolver for PhaseLift's prox (TFOCS/prox_trace.m:88-147: eig((X + X^H)/2), every
// eigenvalue above lambda * step kept; called at every tfocs_AT.m:60 step), d = min(m, n) <= 256.
//
// The one-stage reduction (ace_spectral.hip hetrd_blk_kernel) reads the trailing matrix once per column: d^3 / 6
// entries per matrix, a chain of reductions per column, no matrix cores.  Here (tools/proto_heev2.py is the numpy
// model of the same index conventions):
//
//   he2hb_kernel  stage 1, dense -> band of width 16 (LAPACK zhetrd_he2hb, lower): per panel of 16 columns the
//                 panel below the band is QR-factored (zgeqr2, one panel row per thread in registers, 4 waves),
//                 T = zlarft, V T^H kept for the back-transform, and the trailing matrix takes Q^H A Q as
//                 X = A V T,  W = X - V (T^H V^H X) / 2,  A -= V W^H + W V^H, all 16 x 16 complex tiles on
//                 v_mfma_f64_16x16x4_f64 (4 real products per complex one); the trailing matrix is read twice and
//                 written once per panel (d^3 / 48 entries per pass); two matrices per CU
//   hb2st_kernel  stage 2, band -> real symmetric tridiagonal by bulge chasing (Householder reflectors of length
//                 <= 16; each chase step right-applies the previous reflector to the block below it, annihilates
//                 the first column of the bulge and applies the new reflector to the next diagonal block), the
//                 band in LDS; sweep i runs on wave i mod 8, 2 steps behind sweep i - 1, so that 8 sweeps are in
//                 flight on disjoint footprints (the same arithmetic as one sweep after the other)
//   trieig_kernel (ace_spectral.hip) the eigenpairs of the tridiagonal above tau
//   bt2q2_kernel  back-transform through the stage-2 reflectors: 32 eigenvectors per work-group, each in the
//                 registers of 16 lanes, reflectors applied in a lag-pipelined order that needs no barrier
//   bt2q1_kernel  back-transform through the stage-1 blocks Z -= V ((V T^H)^H Z) on the matrix cores, 32 vectors
//                 per work-group in registers
//
// Matrices whose order is not a multiple of 16 are handled as if zero-padded to dp = 16 ceil(d / 16): the padded
// rows and columns stay exactly zero through stage 1 (masked loads and stores), stage 2 and the tridiagonal run on
// the order d itself.
#include <algorithm>
#include <type_traits>

#include "ace_common.hpp"
#include "ace_host.hpp"
#include "ace_pipe.hpp"

namespace ace {

namespace {

constexpr int H2_MAXD = 256;
// stage 1: 4 waves per matrix, two matrices per CU (LDS 47 KB, <= 256 VGPRs each): one matrix's serial panel QR
// overlaps the other's MFMA phases; wave w owns the trailing matrix's block rows w + 4 h (h < S1_NH)
constexpr int S1_THREADS = 256, S1_NW = S1_THREADS / 64, S1_NH = (H2_MAXD / 16 + S1_NW - 1) / S1_NW;
constexpr int S2_THREADS = 512, S2_NW = S2_THREADS / 64;
// super-steps between consecutive sweeps: step j of sweep i touches rows [s_j, s_j + 16) x columns [s_j - 16, s_j + 16)
// (s_j = i + 1 + 16 j); step j - 2 of sweep i + 1 touches rows [s_j - 31, s_j - 15), disjoint from it, and needs only
// steps <= j - 1 of sweep i (their footprints meet at row s_j - 16), which ran a super-step earlier
constexpr int S2_LAG = 2;
// LDS stride (complex) of a band column: offsets 0..31 (band 16 + bulge) and 2 pad, so that A[r][c] sits at
// (ABS - 1) c + r == c + r (mod 16 complex = the 64 banks): the chase's row-wise and column-wise 16 x 16 block
// accesses both spread over the banks (with 33, c + r became r: 16-way conflicts on the column-wise ones)
constexpr int ABS = 34;

// per-realisation extra scratch (doubles): T of the stage-1 panels [np][16][16], the panel's W [dp][16] and V, V T^H
// of every panel,
// the stage-2 reflectors (v[16], tau) of sweep i, step j at [ts][r][j] with the back-transform's time step
// ts = d - 2 - i + j (q2_index): the 16 step lanes of a time step read 16 consecutive entries per element r
struct H2Lay {
    long long T1, W, V, VT, Q2, stride;
    int dp, np, jm;
};
H2Lay h2lay(int d) {
    H2Lay x{};
    x.dp = (d + 15) & ~15;
    x.np = std::max(0, x.dp / 16 - 1);
    x.jm = x.dp / 16;
    long long o = 0;
    auto take = [&](long long nd) { long long p = o; o += (nd + 31) & ~31LL; return p; };
    x.T1 = take(2LL * std::max(1, x.np) * 256);
    x.W = take(2LL * x.dp * 16);
    x.V = take(2LL * x.dp * 16);   // the stage-1 panel's V [dp][16]
    x.VT = take(2LL * std::max(1, x.np) * x.dp * 16);   // V_p T_p^H per panel [np][dp][16] (rows from the panel's r0)
    x.Q2 = take(2LL * (d + 14) * 17 * 16);
    x.stride = o;
    return x;
}

__host__ __device__ __forceinline__ long long q2_index(int d, int i, int j, int r) {
    return ((long long)(d - 2 - i + j) * 17 + r) * 16 + j;
}
__device__ __forceinline__ d2 cconj(d2 a) { return make_double2(a.x, -a.y); }
__device__ __forceinline__ d2 cneg(d2 a) { return make_double2(-a.x, -a.y); }
__device__ __forceinline__ d2 czero() { return make_double2(0.0, 0.0); }

// lanes of one wave exchanging data through LDS: a wavefront-scope fence orders the accesses for the compiler and
// needs no wait (a wave's LDS operations execute in order), unlike a workgroup-scope one, which would also wait for
// the wave's outstanding global stores
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// a work-group barrier that orders LDS only (an MMRA-restricted fence: waits for the LDS operations, not for the
// wave's global stores, which no other wave of the kernel reads)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// LAPACK zlarfg from (alpha, ||x(2:n)||^2): H^H (alpha; x) = (beta; 0), H = I - tau v v^H, v = (1; x * scal)
struct Refl {
    d2 tau, scal;
    double beta;
};
__device__ __forceinline__ Refl zlarfg_dev(d2 alpha, double xn2) {
    Refl r{czero(), czero(), alpha.x};
    if (!(xn2 == 0.0 && alpha.y == 0.0)) {
        const double beta = -copysign(sqrt(alpha.x * alpha.x + alpha.y * alpha.y + xn2), alpha.x);
        r.beta = beta;
        r.tau = make_double2((beta - alpha.x) / beta, -alpha.y / beta);
        const d2 den = make_double2(alpha.x - beta, alpha.y);   // scal = 1 / (alpha - beta)
        const double dn = 1.0 / cabs2(den);
        r.scal = make_double2(den.x * dn, -den.y * dn);
    }
    return r;
}

// complex 16 x 16 accumulator in the f64 MFMA D layout: lane l, register j holds D[(l >> 4) + 4 j][l & 15];
// operands of k-step s: A lane l = A[l & 15][4 s + (l >> 4)], B lane l = B[4 s + (l >> 4)][l & 15]
struct Cacc {
    d4v r, i;
};
__device__ __forceinline__ Cacc cacc0() {
    Cacc a;
    a.r = d4v{0.0, 0.0, 0.0, 0.0};
    a.i = d4v{0.0, 0.0, 0.0, 0.0};
    return a;
}
__device__ __forceinline__ d4v mfma64(double a, double b, d4v c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void cmma(Cacc& d, d2 a, d2 b) {   // d += a b, one k-step
    d.r = mfma64(a.x, b.x, d.r);
    d.r = mfma64(-a.y, b.y, d.r);
    d.i = mfma64(a.x, b.y, d.i);
    d.i = mfma64(a.y, b.x, d.i);
}
__device__ __forceinline__ d2 cget(const Cacc& a, int j) { return make_double2(a.r[j], a.i[j]); }

__device__ __forceinline__ double row_shr1(double x) {   // lane l <- lane l - 1 within each 16-lane row (lane 0: 0)
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x111, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x111, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double ror8(double x) {   // lane l <- lane l ^ 8 (DPP row_ror:8 inside the 16-lane row)
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x128, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x128, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ d2 quad_sum(d2 v) {   // over the 4 lanes of a quad (DPP, identical in every lane)
    v.x += bfly16<1>(v.x);
    v.y += bfly16<1>(v.y);
    v.x += bfly16<2>(v.x);
    v.y += bfly16<2>(v.y);
    return v;
}

// ---------------------------------------------------------------- stage 1: dense -> band (width 16)
// Per panel p (columns 16 p .., trailing matrix A22 from row / column r0 = 16 p + 16, tt tiles of 16):
//   QR             zgeqr2 of the panel below the band block by all waves, one panel row per thread in registers
//                  (the column loop unrolled; per column two work-group barriers: the norm, the 15 dot products),
//                  then V (unit diagonal) to global scratch, the Gram V^H V on the matrix cores and T (zlarft)
//   X = A22 V T    all waves; wave w owns block rows w + 4 h (row tiles J <= I of A22 and the conjugate transposes
//                  of the column tiles J > I; the diagonal tile made Hermitian), the next tile's operands loaded
//                  while the current one multiplies
//   W = X - V (T^H (V^H X)) / 2
//   A22 -= V W^H + W V^H on the lower tiles
// Two matrices per CU (LDS 46 KB, <= 256 VGPRs per work-group): one's barrier-bound QR overlaps the other's
// matrix-core phases.
constexpr int TBS = 9;   // LDS row stride of a wave's transposed partial sums (8 columns)

struct QrLds {
    d2 tb[S1_NW][64 * TBS];   // per wave: the column dot products' partials, transposed (aliased by the X / M slots)
    d2 wpart[S1_NW][16];      // per wave: its sums of the dot products
    d2 twv[S1_NW][16];        // per wave: its copy of conj(tau) w
    d2 sG[256], s_tau[16], s_alpha;
    double red[S1_NW];
};
static_assert(64 * TBS >= 256, "a wave's X / M slot must fit its tb");

// zgeqr2 of the panel A[r0 .. dp)[k .. k + 16) (thread t holds row r0 + t), V (unit diagonal, zeros above) into Vg,
// the panel (R, beta, reflectors) back into C, T (zlarft from the Gram) into sT and T1p.  Ends with a barrier.
__device__ __forceinline__ void panel_qr(int d, int k, int r0, int dp, d2* C, d2* Vg, d2* T1p, d2* sT, QrLds& q) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, lr = lane >> 4, lc = lane & 15;
    const int L = dp - r0, tt = L >> 4, rr = t, r = r0 + rr;
    d2 P[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {   // (unconditional loads from clamped addresses, then masked: see ldC)
        const d2 x = C[(long long)min(r, d - 1) * d + min(k + c, d - 1)];
        P[c] = (rr < L && r < d && k + c < d) ? x : czero();
    }
    d2* tbw = q.tb[w];
    // (one call per column with j a compile-time constant: the register array P is indexed by constants only)
    auto col_step = [&](auto jc) {
        constexpr int j = decltype(jc)::value;
        double s = wave_sum_dpp(rr > j ? cabs2(P[j]) : 0.0);   // (rows >= L hold zeros)
        if (lane == 0) q.red[w] = s;
        if (t == j) q.s_alpha = P[j];
        lds_barrier();
        s = 0.0;
#pragma unroll
        for (int ww = 0; ww < S1_NW; ++ww) s += q.red[ww];
        const Refl R = zlarfg_dev(q.s_alpha, s);
        const d2 v = rr > j ? cmul(P[j], R.scal) : make_double2(rr == j ? 1.0 : 0.0, 0.0);
        // w_c = v^H P[.][c] (c > j): the wave's partials transposed through LDS in halves of 8 columns (lane
        // (part, c8) adds 8 lanes' partials of column c8, three shuffles the 8 parts), then the waves' sums
        if (j < 15) {
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                if (8 * hf + 7 <= j) continue;
#pragma unroll
                for (int c8 = 0; c8 < 8; ++c8) {
                    const int c = 8 * hf + c8;
                    tbw[lane * TBS + c8] = c > j ? cmulc(v, P[c]) : czero();
                }
                wave_sync();
                const int part = lane >> 3, c8 = lane & 7;
                d2 a = czero();
#pragma unroll
                for (int l = 0; l < 8; ++l) a = cadd(a, tbw[(8 * part + l) * TBS + c8]);
                a.x += ror8(a.x);   // (the 8 parts: lanes ^ 8, ^ 16, ^ 32)
                a.y += ror8(a.y);
                a.x = xor32_sum(xor16_sum(a.x));
                a.y = xor32_sum(xor16_sum(a.y));
                if (part == 0) q.wpart[w][8 * hf + c8] = a;
                wave_sync();
            }
            lds_barrier();
            if (lane < 16) {   // (lane c of every wave: conj(tau) w_c into the wave's copy)
                d2 a = czero();
#pragma unroll
                for (int ww = 0; ww < S1_NW; ++ww) a = cadd(a, q.wpart[ww][lane]);
                q.twv[w][lane] = cmul(cconj(R.tau), a);
            }
            wave_sync();
#pragma unroll
            for (int c = j + 1; c < 16; ++c) P[c] = csub(P[c], cmul(v, q.twv[w][c]));   // (I - conj(tau) v v^H)
        }
        P[j] = rr == j ? make_double2(R.beta, 0.0) : (rr > j ? v : P[j]);   // rows < j: R
        if (t == 0) q.s_tau[j] = R.tau;
    };
    using std::integral_constant;
    col_step(integral_constant<int, 0>{});
    col_step(integral_constant<int, 1>{});
    col_step(integral_constant<int, 2>{});
    col_step(integral_constant<int, 3>{});
    col_step(integral_constant<int, 4>{});
    col_step(integral_constant<int, 5>{});
    col_step(integral_constant<int, 6>{});
    col_step(integral_constant<int, 7>{});
    col_step(integral_constant<int, 8>{});
    col_step(integral_constant<int, 9>{});
    col_step(integral_constant<int, 10>{});
    col_step(integral_constant<int, 11>{});
    col_step(integral_constant<int, 12>{});
    col_step(integral_constant<int, 13>{});
    col_step(integral_constant<int, 14>{});
    col_step(integral_constant<int, 15>{});
    // the panel back into C, V into Vg (rows < L)
    if (rr < L) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            if (r < d && k + c < d) C[(long long)r * d + k + c] = P[c];
            Vg[rr * 16 + c] = rr > c ? P[c] : make_double2(rr == c ? 1.0 : 0.0, 0.0);
        }
    }
    __syncthreads();   // (Vg: global stores read by the other waves)
    // the Gram V^H V: wave w's tiles I = w (mod S1_NW), partials summed through LDS (rows of tile I: lane (lr + 4 q, lc))
    Cacc G = cacc0();
    for (int I = w; I < tt; I += S1_NW) {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            const d2 vv = Vg[(16 * I + lr + 4 * qq) * 16 + lc];
            cmma(G, cconj(vv), vv);
        }
    }
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) tbw[(lr + 4 * j4) * 16 + lc] = cget(G, j4);
    lds_barrier();
    if (w == 0) {
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
            const int e = (lr + 4 * j4) * 16 + lc;
            d2 a = czero();
#pragma unroll
            for (int ww = 0; ww < S1_NW; ++ww) a = cadd(a, q.tb[ww][e]);
            q.sG[e] = a;
        }
        wave_sync();
        if (lane < 16) {   // zlarft (forward, columnwise): lane a computes row a of T
            const int a = lane;
            d2 Tr[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const d2 ti = q.s_tau[i];
                d2 acc = czero();
#pragma unroll
                for (int c = 0; c < 16; ++c)
                    if (c < i && c >= a) acc = cadd(acc, cmul(Tr[c], cneg(cmul(ti, q.sG[c * 16 + i]))));
                Tr[i] = i == a ? ti : (i > a ? acc : czero());
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                sT[a * 16 + i] = Tr[i];
                T1p[a * 16 + i] = Tr[i];
            }
        }
    }
    lds_barrier();
}

__global__ __launch_bounds__(S1_THREADS) __attribute__((amdgpu_waves_per_eu(2))) void he2hb_kernel(int d, double* scratch, HeevLayout hl, double* xs, H2Lay xl,
                                                           const int* active) {
    const int b = blockIdx.x;
    if (active && !active[b]) return;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, lr = lane >> 4, lc = lane & 15;
    d2* C = reinterpret_cast<d2*>(scratch + (long long)b * hl.stride + hl.C);
    double* xb = xs + (long long)b * xl.stride;
    d2* T1 = reinterpret_cast<d2*>(xb + xl.T1);
    d2* Wg = reinterpret_cast<d2*>(xb + xl.W);
    d2* Vg2 = reinterpret_cast<d2*>(xb + xl.V);
    d2* VTg = reinterpret_cast<d2*>(xb + xl.VT);
    const int dp = xl.dp;
    __shared__ QrLds q;
    __shared__ d2 sT[256];
    d2* slw = q.tb[w];   // the wave's X / M slot (its QR partials' space)
    // (loads unconditional from a clamped address, then masked: no branch around a load, so that a tile's loads
    // issue together instead of one wait each)
    auto ldC = [&](int r, int c) -> d2 {
        const d2 v = C[(long long)min(r, d - 1) * d + min(c, d - 1)];
        return (r < d && c < d) ? v : czero();
    };
    auto stC = [&](int r, int c, d2 v) {
        if (r < d && c < d) C[(long long)r * d + c] = v;
    };
#ifdef ACE_H2_STAMPS
    unsigned long long st_ph[4] = {0, 0, 0, 0}, st_t = __builtin_amdgcn_s_memrealtime();
    auto stamp = [&](int ph) {
        const unsigned long long n = __builtin_amdgcn_s_memrealtime();
        st_ph[ph] += n - st_t;
        st_t = n;
    };
#else
    auto stamp = [](int) {};
#endif
    for (int p = 0; p < xl.np; ++p) {
        const int r0 = 16 * p + 16, tt = (dp - r0) >> 4;
        const d2* Vg = Vg2;
        panel_qr(d, 16 * p, r0, dp, C, Vg2, T1 + p * 256, sT, q);
        {   // V T^H for the back-transform (Z -= V ((V T^H)^H Z): no per-work-group T product there), tile I of
            // the panel's rows on wave I mod 4: D[i][c] = sum_k V[16 I + i][k] conj(T[c][k])
            d2* VTp = VTg + (long long)p * dp * 16;
            for (int I = w; I < tt; I += S1_NW) {
                Cacc D = cacc0();
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    cmma(D, Vg[(16 * I + lc) * 16 + 4 * s + lr], cconj(sT[lc * 16 + 4 * s + lr]));
#pragma unroll
                for (int j4 = 0; j4 < 4; ++j4) VTp[(16 * I + lr + 4 * j4) * 16 + lc] = cget(D, j4);
            }
        }
        stamp(0);
        // ---- X = A22 V T for the wave's block rows I = w + 4 h, XG of them at once per block column J (the
        // tiles' operand loads of one J in flight together: the phase is bound by memory round trips)
        // (X goes to Wg tile by tile, W is formed in place; M = V^H X accumulates as the tiles come)
        auto lda = [&](int I, int J, int s) -> d2 {   // A22 tile (I, J) from the lower triangle (branch-free)
            const int ri = r0 + 16 * I, rj = r0 + 16 * J, c = 4 * s + lr;
            const bool below = J < I || (J == I && lc >= c);
            d2 x = ldC(below ? ri + lc : rj + c, below ? rj + c : ri + lc);
            x.y = below ? (J == I && lc == c ? 0.0 : x.y) : -x.y;
            return x;
        };
        Cacc Mp = cacc0();
        constexpr int XG = 2;   // block rows per pass (registers: XG accumulators and XG x 4 operands)
        for (int h0 = 0; h0 < S1_NH; h0 += XG) {
            if (w + S1_NW * h0 >= tt) break;
            Cacc Y[XG];
#pragma unroll
            for (int h = 0; h < XG; ++h) Y[h] = cacc0();
            // operands of block column J + 1 loaded while J multiplies (the last round re-loads J: clamped index,
            // no conditional load)
            d2 bv[4], a[XG][4];
            auto load_j = [&](int J, d2 (&bo)[4], d2 (&ao)[XG][4]) {
#pragma unroll
                for (int s = 0; s < 4; ++s) bo[s] = Vg[(16 * J + 4 * s + lr) * 16 + lc];
#pragma unroll
                for (int h = 0; h < XG; ++h) {
                    const int I = w + S1_NW * (h0 + h);
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        const d2 x = lda(min(I, tt - 1), J, s);
                        ao[h][s] = I < tt ? x : czero();
                    }
                }
            };
            load_j(0, bv, a);
            for (int J = 0; J < tt; ++J) {
                d2 bn[4], an[XG][4];
                load_j(min(J + 1, tt - 1), bn, an);
#pragma unroll
                for (int h = 0; h < XG; ++h)
                    if (w + S1_NW * (h0 + h) < tt) {
#pragma unroll
                        for (int s = 0; s < 4; ++s) cmma(Y[h], a[h][s], bv[s]);
                    }
#pragma unroll
                for (int s = 0; s < 4; ++s) bv[s] = bn[s];
#pragma unroll
                for (int h = 0; h < XG; ++h)
#pragma unroll
                    for (int s = 0; s < 4; ++s) a[h][s] = an[h][s];
            }
#pragma unroll
            for (int h = 0; h < XG; ++h) {
                const int I = w + S1_NW * (h0 + h);
                if (I >= tt) continue;
#pragma unroll
                for (int j4 = 0; j4 < 4; ++j4) slw[(lr + 4 * j4) * 17 + lc] = cget(Y[h], j4);   // (row stride 17:
                wave_sync();                                                                      // the transposed read)
                Cacc Xh = cacc0();
#pragma unroll
                for (int s = 0; s < 4; ++s) cmma(Xh, slw[lc * 17 + 4 * s + lr], sT[(4 * s + lr) * 16 + lc]);
                wave_sync();
#pragma unroll
                for (int j4 = 0; j4 < 4; ++j4) Wg[(16 * I + lr + 4 * j4) * 16 + lc] = cget(Xh, j4);
#pragma unroll
                for (int s = 0; s < 4; ++s) cmma(Mp, cconj(Vg[(16 * I + 4 * s + lr) * 16 + lc]), cget(Xh, s));
            }
        }
        stamp(1);
        // ---- M = V^H X (partials per wave, summed in wave order), S = T^H M, W = X - V S / 2
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) slw[(lr + 4 * j4) * 16 + lc] = cget(Mp, j4);
        lds_barrier();
        Cacc S = cacc0();
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int kk = 4 * s + lr;
            d2 m = czero();
#pragma unroll
            for (int ww = 0; ww < S1_NW; ++ww) m = cadd(m, q.tb[ww][kk * 16 + lc]);
            cmma(S, cconj(sT[kk * 16 + lc]), m);
        }
#pragma unroll
        for (int h = 0; h < S1_NH; ++h) {
            const int I = w + S1_NW * h;
            if (I >= tt) continue;
            Cacc U = cacc0();
#pragma unroll
            for (int s = 0; s < 4; ++s) cmma(U, Vg[(16 * I + lc) * 16 + 4 * s + lr], cget(S, s));
#pragma unroll
            for (int j4 = 0; j4 < 4; ++j4) {   // (the thread's own X entries)
                d2& x = Wg[(16 * I + lr + 4 * j4) * 16 + lc];
                x = csub(x, cscale(cget(U, j4), 0.5));
            }
        }
        __syncthreads();
        stamp(2);
        // ---- A22 -= V W^H + W V^H on the lower tiles: wave w takes the block rows of snake order (I mod 8 = w or
        // 7 - w: equal tile counts per wave), two rows at a time with both rows' tiles of one J loaded together
        for (int pr = 0; pr < 2; ++pr) {
            const int Ia = 8 * pr + w, Ib = 8 * pr + 7 - w;   // (Ia < Ib)
            if (Ia >= tt) break;
            const bool hb = Ib < tt;
            d2 va[4], wa[4], vb2[4], wb2[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int c = 4 * s + lr;
                va[s] = Vg[(16 * Ia + lc) * 16 + c];
                wa[s] = Wg[(16 * Ia + lc) * 16 + c];
                vb2[s] = Vg[(16 * min(Ib, tt - 1) + lc) * 16 + c];   // (unused unless hb)
                wb2[s] = Wg[(16 * min(Ib, tt - 1) + lc) * 16 + c];
            }
            const int Jn = hb ? Ib : Ia;
            for (int J = 0; J <= Jn; ++J) {
                const int rj = r0 + 16 * J;
                const bool ta = J <= Ia;
                d2 wj[4], vj[4];
                Cacc A0, A1;
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int c = 4 * s + lr;
                    wj[s] = Wg[(16 * J + lc) * 16 + c];
                    vj[s] = Vg[(16 * J + lc) * 16 + c];
                }
#pragma unroll
                for (int j4 = 0; j4 < 4; ++j4) {
                    const d2 x0 = ldC(r0 + 16 * Ia + lr + 4 * j4, rj + lc);   // (used if ta)
                    const d2 x1 = ldC(r0 + 16 * Ib + lr + 4 * j4, rj + lc);   // (used if hb)
                    A0.r[j4] = x0.x;
                    A0.i[j4] = x0.y;
                    A1.r[j4] = x1.x;
                    A1.i[j4] = x1.y;
                }
                if (ta) {
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        cmma(A0, cneg(va[s]), cconj(wj[s]));
                        cmma(A0, cneg(wa[s]), cconj(vj[s]));
                    }
#pragma unroll
                    for (int j4 = 0; j4 < 4; ++j4) stC(r0 + 16 * Ia + lr + 4 * j4, rj + lc, cget(A0, j4));
                }
                if (hb) {
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        cmma(A1, cneg(vb2[s]), cconj(wj[s]));
                        cmma(A1, cneg(wb2[s]), cconj(vj[s]));
                    }
#pragma unroll
                    for (int j4 = 0; j4 < 4; ++j4) stC(r0 + 16 * Ib + lr + 4 * j4, rj + lc, cget(A1, j4));
                }
            }
        }
        __syncthreads();
        stamp(3);
    }
#ifdef ACE_H2_STAMPS
    if (t == 0 && (b % 101) == 0)
        printf("he2hb b %d: qr %llu X %llu W %llu upd %llu (x10ns)\n", b, st_ph[0], st_ph[1], st_ph[2], st_ph[3]);
#endif
}

// ---------------------------------------------------------------- stage 2: band -> tridiagonal
__global__ __launch_bounds__(S2_THREADS) void hb2st_kernel(int d, double* scratch, HeevLayout hl, double* xs, H2Lay xl,
                                                           const int* active) {
    const int b = blockIdx.x;
    if (active && !active[b]) return;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, lq = lane >> 2, lm = lane & 3;
    double* base = scratch + (long long)b * hl.stride;
    const d2* C = reinterpret_cast<const d2*>(base + hl.C);
    d2* Q2 = reinterpret_cast<d2*>(xs + (long long)b * xl.stride + xl.Q2);
    extern __shared__ double smem[];
    d2* AB = reinterpret_cast<d2*>(smem);   // AB[c * ABS + o] = A[c + o][c], o < 32
    __shared__ d2 vb[S2_NW][16], wb[S2_NW][16];
    for (int e = t; e < d * 32; e += S2_THREADS) {
        const int c = e >> 5, o = e & 31;
        d2 v = czero();
        if (o <= 16 && c + o < d) {
            v = C[(long long)(c + o) * d + c];
            if (o == 0) v.y = 0.0;
        }
        AB[c * ABS + o] = v;
    }
    __syncthreads();
#ifdef ACE_H2_STAMPS
    unsigned long long hs[4] = {0, 0, 0, 0}, hs_t = __builtin_amdgcn_s_memtime();
    auto hstamp = [&](int ph) {
        const unsigned long long n = __builtin_amdgcn_s_memtime();
        hs[ph] += n - hs_t;
        hs_t = n;
    };
#else
    auto hstamp = [](int) {};
#endif
    auto at = [&](int r, int c) -> d2& { return AB[c * ABS + (r - c)]; };   // r >= c
    // a read at a clamped (always valid) address, masked afterwards: no branch around the LDS load, so that a
    // step's reads issue together instead of one wait each
    auto atm = [&](int r, int c, bool ok) -> d2 {
        const d2 x = AB[min(c, d - 1) * ABS + min(max(r - c, 0), ABS - 1)];
        return ok ? x : czero();
    };
    auto herm = [&](int r, int c) -> d2 {   // (one LDS read whatever the lane's side of the diagonal)
        const int lo = min(r, c);
        d2 a = AB[lo * ABS + abs(r - c)];
        a.y = r > c ? a.y : (r < c ? -a.y : 0.0);
        return a;
    };
    // D <- H^H D H on the diagonal block [r0, r0 + len) with v in vb[w] and the lane's entries v[lm + 4 u] in vr
    // (zhetd2's x, w, rank-2 update); lane (row lq, columns lm + 4 u)
    d2 vr[4];
    auto two_sided = [&](int r0, int len, d2 tau) {
        d2 xr = czero();
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int cc = lm + 4 * u;
            const d2 hv = herm(min(r0 + lq, d - 1), min(r0 + cc, d - 1));
            if (lq < len && cc < len) xr = cadd(xr, cmul(hv, vr[u]));
        }
        xr = cmul(tau, quad_sum(xr));
        d2 vq = vb[w][lq];
        if (lq >= len) vq = czero();
        d2 pr = (lm == 0 && lq < len) ? cmulc(xr, vq) : czero();
        pr.x = wave_sum_dpp(pr.x);
        pr.y = wave_sum_dpp(pr.y);
        const d2 al = cscale(cmul(tau, pr), -0.5);
        const d2 wr = cadd(xr, cmul(al, vq));
        if (lm == 0) wb[w][lq] = wr;
        wave_sync();
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int cc = lm + 4 * u;
            const d2 av = atm(r0 + lq, r0 + cc, true);   // (unconditional reads, conditional store)
            d2 x = csub(av, cadd(cmul(vq, cconj(wb[w][cc])), cmul(wr, cconj(vr[u]))));
            if (cc == lq) x.y = 0.0;
            if (lq < len && cc <= lq) at(r0 + lq, r0 + cc) = x;
        }
        wave_sync();
    };
    d2 tau = czero();
    int r0 = 0, len = 0;
    const int nss = S2_LAG * (d - 2) + 16;
    static_assert(S2_NW * S2_LAG >= 16, "a wave's next sweep must start after its current one (16 steps at most)");
    for (int ss = 0; ss < nss; ++ss) {
        int i = -1, j = 0;
        if (ss >= S2_LAG * w) {
            i = w + S2_NW * ((ss - S2_LAG * w) / (S2_LAG * S2_NW));
            j = ss - S2_LAG * i;
        }
        if (i >= 0 && i < d - 1 && j < (d - 1 - i + 15) / 16) {   // (uniform per wave)
            auto slot = [&](int r) -> d2& { return Q2[q2_index(d, i, j, r)]; };
            if (j == 0) {
                // the sweep's first reflector: column i below the subdiagonal
                r0 = i + 1;
                len = min(16, d - 1 - i);
                const d2 x = lq < len ? AB[i * ABS + 1 + lq] : czero();
                double s = (lm == 0 && lq >= 1 && lq < len) ? cabs2(x) : 0.0;
                s = wave_sum_dpp(s);
                const Refl R = zlarfg_dev(AB[i * ABS + 1], s);
                tau = R.tau;
                const d2 v = lq == 0 ? make_double2(1.0, 0.0) : (lq < len ? cmul(x, R.scal) : czero());
                wave_sync();
                if (lm == 0) {
                    vb[w][lq] = v;
                    if (lq < len) AB[i * ABS + 1 + lq] = lq == 0 ? make_double2(R.beta, 0.0) : czero();
                    slot(lq) = v;
                    if (lq == 0) slot(16) = tau;
                }
                wave_sync();
#pragma unroll
                for (int u = 0; u < 4; ++u) vr[u] = vb[w][lm + 4 * u];
                two_sided(r0, len, tau);
            } else {
                const int s0 = r0 + len, len2 = min(16, d - s0);
                // right-apply the previous reflector to the block below it: Bk = A[s0 .. s0 + len2)[r0 .. r0 + len)
                // (lane: row lq, columns lm + 4 u)
                d2 bk[4];
                d2 y = czero();
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int cc = lm + 4 * u;
                    bk[u] = atm(s0 + lq, r0 + cc, lq < len2 && cc < len);
                    y = cadd(y, cmul(bk[u], vr[u]));   // (the previous reflector's entries, kept in registers)
                }
                y = cmul(tau, quad_sum(y));
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int cc = lm + 4 * u;
                    if (lq < len2 && cc < len) at(s0 + lq, r0 + cc) = csub(bk[u], cmul(y, cconj(vr[u])));
                }
                wave_sync();
                hstamp(0);
                // the bulge's first column -> the new reflector, applied from the left to the block (lane: column
                // lq, rows lm + 4 u)
                d2 xc[4], bc[4];
                double s = 0.0;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int rr = lm + 4 * u;
                    xc[u] = atm(s0 + rr, r0, rr < len2);
                    if (rr >= 1) s += cabs2(xc[u]);
                    bc[u] = atm(s0 + rr, r0 + lq, rr < len2 && lq < len);
                }
                s += bfly16<1>(s);
                s += bfly16<2>(s);
                const Refl R = zlarfg_dev(at(s0, r0), s);
                d2 v2[4];
                d2 ws = czero();
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int rr = lm + 4 * u;
                    v2[u] = rr == 0 ? make_double2(1.0, 0.0) : (rr < len2 ? cmul(xc[u], R.scal) : czero());
                    ws = cadd(ws, cmulc(v2[u], bc[u]));
                }
                ws = quad_sum(ws);
                const d2 ctw = cmul(cconj(R.tau), ws);
                wave_sync();
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int rr = lm + 4 * u;
                    if (rr < len2 && lq < len)
                        at(s0 + rr, r0 + lq) = lq == 0 ? make_double2(rr == 0 ? R.beta : 0.0, 0.0)
                                                       : csub(bc[u], cmul(v2[u], ctw));
                    if (lq == 0) {
                        vb[w][rr] = v2[u];
                        slot(rr) = v2[u];
                    }
                }
                if (lane == 0) slot(16) = R.tau;
#pragma unroll
                for (int u = 0; u < 4; ++u) vr[u] = v2[u];   // (rows lm + 4 u: the layout two_sided reads)
                tau = R.tau;
                r0 = s0;
                len = len2;
                wave_sync();
                hstamp(1);
                two_sided(r0, len, tau);
                hstamp(2);
            }
        }
        lds_barrier();   // (the Q2 slots are global stores read only by bt2q2_kernel)
        hstamp(3);
    }
#ifdef ACE_H2_STAMPS
    if (t == 0 && (b % 101) == 0)
        printf("hb2st b %d: %d super-steps, wave 0 cycles: right %llu left %llu two-sided %llu barrier %llu\n", b, nss,
               hs[0], hs[1], hs[2], hs[3]);
#endif
    double* dd = base + hl.dd;
    double* ee = base + hl.ee;
    for (int i = t; i < d; i += S2_THREADS) {
        dd[i] = AB[i * ABS].x;
        ee[i] = i + 1 < d ? AB[i * ABS + 1].x : 0.0;
    }
}

// ---------------------------------------------------------------- back-transform: V = Q1 Q2 z
// 1-D grids map work-group g -> (matrix, chunk of vectors) with all chunks of a matrix on one XCD (g mod 8), so that
// they share the matrix's reflectors in that XCD's L2.
__device__ __forceinline__ void bt_decode(int g, int nc, int& b, int& c) {
    const int lb = g & 7, rest = g >> 3;
    c = rest % nc;
    b = (rest / nc) * 8 + lb;
}

// Q2 = prod_i prod_j H_ij (sweep i ascending; a sweep's reflectors act on the disjoint rows i + 1 + 16 j ..), applied
// last sweep first.  Lane (vector, j) of a wave applies step j's reflector of sweep i = d - 2 - ts + j at time step
// ts: two reflectors whose rows overlap keep their order (sweep i before i' < i: j - j' < i - i' whenever they
// overlap) and two of one time step never overlap.  Each vector lives in the registers of its 16 step lanes: lane
// j holds the 16 rows of its window [i + 1 + 16 j, i + 16 + 16 j] and the row below it (the gap to lane j + 1's
// window).  Every time step moves the windows up by one row: lane j's new top row is lane j - 1's gap row (DPP
// row_shr:1 inside the 16-lane row), lane 0's the next untouched row of z, and the bottom row becomes the gap.  The
// window index rotates through the registers (the time loop is unrolled by 16).  A lane writes its rows out after
// its last reflector (sweep 0): they are final then (every later reflector of the schedule lies below them).
// The work-group's 8 waves (32 vectors) share the reflectors, staged in LDS 16 time steps at a time (the layout
// q2_index makes a time step's reflectors contiguous), double-buffered, one barrier pair per 16 time steps.
constexpr int Q2_THREADS = 512, Q2_NV = Q2_THREADS / 16, Q2_BLK = 16;   // (252 VGPRs: 2 waves per SIMD; LDS 136 KB)
constexpr int Q2_BLKE = Q2_BLK * 17 * 16;   // staged entries (complex) per block of time steps
__global__ __launch_bounds__(Q2_THREADS) void bt2q2_kernel(int d, int kmax, int batch, int nc, const double* scratch,
                                                           HeevLayout hl, const double* xs, H2Lay xl, double* Vout,
                                                           const int* active) {
    int b, c;
    bt_decode(blockIdx.x, nc, b, c);
    if (b >= batch || (active && !active[b])) return;
    const double* base = scratch + (long long)b * hl.stride;
    const int k = (int)base[hl.misc];
    const int q0 = c * Q2_NV;
    if (q0 >= k) return;
    const int t = threadIdx.x, lane = t & 63, j = lane & 15, qv = (t >> 4);
    __shared__ d2 vs[2][Q2_BLKE];
    const d2* Q2 = reinterpret_cast<const d2*>(xs + (long long)b * xl.stride + xl.Q2);
    const int nt = d - 2 + 16;                       // lane 15's last step is at d - 2 + 15
    const int nblk = (nt + Q2_BLK - 1) / Q2_BLK;
    const long long q2n = (long long)(d + 14) * 17 * 16;   // entries of the layout
    constexpr int PF = (Q2_BLKE + Q2_THREADS - 1) / Q2_THREADS;
    d2 pf[PF];
    auto fetch = [&](int blk) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const long long e = (long long)blk * Q2_BLKE + t + u * Q2_THREADS;
            pf[u] = (t + u * Q2_THREADS < Q2_BLKE && e < q2n) ? Q2[e] : czero();
        }
    };
    auto stage = [&](int buf) {
#pragma unroll
        for (int u = 0; u < PF; ++u)
            if (t + u * Q2_THREADS < Q2_BLKE) vs[buf][t + u * Q2_THREADS] = pf[u];
    };
    fetch(0);
    stage(0);
    if (nblk > 1) fetch(1);
    lds_barrier();
    const bool has_vec = q0 + qv < k;
    const double* zv = base + hl.z + (long long)(q0 + qv) * d;
    d2* vo = reinterpret_cast<d2*>(Vout) + ((long long)b * kmax + q0 + qv) * d;
    d2 win[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) win[u] = czero();
    if (j == 0 && has_vec) {
        win[0] = make_double2(zv[d - 1], 0.0);
        vo[0] = make_double2(zv[0], 0.0);   // (row 0: no reflector touches it)
    }
    d2 gap = czero();
    double zin = 0.0, zin_next = (has_vec && d - 2 - j >= 0) ? zv[d - 2 - j] : 0.0;
    // one block of Q2_BLK time steps from the staged buffer; MOFF = (ts mod 16) of its first step, a compile-time
    // constant so that the window rotation stays in registers (the blocks run in pairs)
    auto run_block = [&](int blk, auto moff_c) {
        constexpr int MOFF = decltype(moff_c)::value;
        const d2* vb = vs[blk & 1];
        if (MOFF % 16 == 0) {   // the next 16 untouched rows of z, d - 2 - t0 - j, one per lane of the group (loaded
                                // a 16-step period ahead)
            zin = zin_next;
            const int zr = d - 2 - (blk + 16 / Q2_BLK) * Q2_BLK - j;
            zin_next = (has_vec && zr >= 0) ? zv[zr] : 0.0;
        }
#pragma unroll
        for (int m = 0; m < Q2_BLK; ++m) {
            const int mm = MOFF + m;                 // ts mod 16
            const int ts = blk * Q2_BLK + m;
            const int i = d - 2 - ts + j;
            const d2* v = vb + m * 17 * 16 + j;
            // the step's reflector, all 17 entries issued together (one LDS round trip per step, not 17)
            d2 vv[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) vv[u] = v[u * 16];
            const d2 tv = v[16 * 16];
            if (i >= 0 && i + 1 + 16 * j < d && ts < nt && !(tv.x == 0.0 && tv.y == 0.0)) {
                d2 dt[4] = {czero(), czero(), czero(), czero()};
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const d2 z = win[(u - mm) & 15];
                    dt[u & 3].x = fma(vv[u].x, z.x, fma(vv[u].y, z.y, dt[u & 3].x));
                    dt[u & 3].y = fma(vv[u].x, z.y, fma(-vv[u].y, z.x, dt[u & 3].y));
                }
                const d2 f = cmul(tv, cadd(cadd(dt[0], dt[1]), cadd(dt[2], dt[3])));
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    d2& z = win[(u - mm) & 15];
                    z.x = fma(-f.x, vv[u].x, fma(f.y, vv[u].y, z.x));
                    z.y = fma(-f.x, vv[u].y, fma(-f.y, vv[u].x, z.y));
                }
            }
            if (i == 0 && has_vec) {   // the lane's last reflector: rows 1 + 16 j .. are final
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int row = 1 + 16 * j + u;
                    if (row < d) vo[row] = win[(u - mm) & 15];
                }
            }
            // shift: the new top row from lane j - 1's gap (lane 0: z), the bottom row becomes the gap
            const double nz = __shfl(zin, (lane & 48) | (mm & 15), 64);
            d2 top = make_double2(row_shr1(gap.x), row_shr1(gap.y));
            if (j == 0) top = make_double2(nz, 0.0);
            gap = win[(15 - mm) & 15];
            win[(15 - mm) & 15] = top;
            __builtin_amdgcn_sched_barrier(0);   // (no hoisting of later steps' LDS reads: they would not fit)
        }
        if (blk + 1 < nblk) {
            lds_barrier();   // (every wave is done with the buffer the next-but-one block goes to)
            stage((blk + 1) & 1);
            if (blk + 2 < nblk) fetch(blk + 2);
            lds_barrier();   // (LDS only: a full barrier would wait for the prefetch just issued)
        }
    };
    for (int blk = 0; blk < nblk; blk += 2) {
        run_block(blk, std::integral_constant<int, 0>{});
        if (blk + 1 < nblk) run_block(blk + 1, std::integral_constant<int, Q2_BLK>{});
    }
}

// Q1 = prod_p (I - V_p T_p V_p^H), the last panel first, on 32 vectors per work-group held in registers in the f64
// MFMA layout (wave w: row tiles w and w + 8, both 16-vector column tiles); W2 = (V_p T_p^H)^H Z (he2hb stored
// V_p T_p^H) is summed over the waves in wave order through LDS, then Z -= V_p W2.  A panel's V operands (both layouts) are loaded for the next panel while the current one
// computes.
constexpr int Q1_THREADS = 512, Q1_NW = 8, Q1_NV = 32;
__global__ __launch_bounds__(Q1_THREADS) void bt2q1_kernel(int d, int kmax, int batch, int nc, const double* scratch,
                                                           HeevLayout hl, const double* xs, H2Lay xl, double* Vout,
                                                           const int* active) {
    int b, c;
    bt_decode(blockIdx.x, nc, b, c);
    if (b >= batch || (active && !active[b])) return;
    const double* base = scratch + (long long)b * hl.stride;
    const int k = (int)base[hl.misc];
    const int q0 = c * Q1_NV;
    if (q0 >= k) return;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, lr = lane >> 4, lc = lane & 15;
    const int dp = xl.dp, nti = dp >> 4;
    __shared__ d2 sl[Q1_NW][2][256];
    const d2* Cm = reinterpret_cast<const d2*>(base + hl.C);
    const d2* VT = reinterpret_cast<const d2*>(xs + (long long)b * xl.stride + xl.VT);
    d2* Vo = reinterpret_cast<d2*>(Vout) + (long long)b * kmax * d;
    Cacc Z[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int cv = 0; cv < 2; ++cv) {
            Z[h][cv] = cacc0();
            const int I = w + Q1_NW * h, q = q0 + 16 * cv + lc;
            if (I >= nti) continue;
#pragma unroll
            for (int j4 = 0; j4 < 4; ++j4) {
                const int row = 16 * I + lr + 4 * j4;
                const d2 z = (q < k && row < d) ? Vo[(long long)q * d + row] : czero();
                Z[h][cv].r[j4] = z.x;
                Z[h][cv].i[j4] = z.y;
            }
        }
    auto vget = [&](int p, int row, int a) -> d2 {   // V_p[row][a] (absolute row): unit diagonal at row 16 p + 16 + a
        const int rr = row - (16 * p + 16);
        if (rr < a || row >= d || p < 0) return czero();
        if (rr == a) return make_double2(1.0, 0.0);
        return Cm[(long long)row * d + 16 * p + a];
    };
    // operands of panel p for the wave's tiles: va (W1: conj V[16 I + 4 s + lr][lc]), vb (U: V[16 I + lc][4 s + lr])
    d2 va[2][4], vb[2][4];
    auto load_v = [&](int p, bool a, bool bb) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int I = w + Q1_NW * h;
            const bool live = p >= 0 && I >= p + 1 && I < nti;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                if (a) va[h][s] = live ? cconj(VT[((long long)p * dp + 16 * (I - p - 1) + 4 * s + lr) * 16 + lc]) : czero();
                if (bb) vb[h][s] = live ? vget(p, 16 * I + lc, 4 * s + lr) : czero();
            }
        }
    };
    load_v(xl.np - 1, true, true);
    for (int p = xl.np - 1; p >= 0; --p) {
        Cacc W1[2] = {cacc0(), cacc0()};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int I = w + Q1_NW * h;
            if (I < p + 1 || I >= nti) continue;
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int cv = 0; cv < 2; ++cv) cmma(W1[cv], va[h][s], cget(Z[h][cv], s));
        }
#pragma unroll
        for (int cv = 0; cv < 2; ++cv)
#pragma unroll
            for (int j4 = 0; j4 < 4; ++j4) sl[w][cv][(lr + 4 * j4) * 16 + lc] = cget(W1[cv], j4);
        lds_barrier();
        // W2 = (V T^H)^H Z = T V^H Z, summed over the waves in wave order (row 4 s + lr of W2 in register s); two
        // waves' partials per round (all 64 loads at once would not fit the registers)
        d2 w2[2][4];
#pragma unroll
        for (int cv = 0; cv < 2; ++cv)
#pragma unroll
            for (int s = 0; s < 4; ++s) w2[cv][s] = czero();
#pragma unroll 2
        for (int ww = 0; ww < Q1_NW; ++ww) {
#pragma unroll
            for (int cv = 0; cv < 2; ++cv)
#pragma unroll
                for (int s = 0; s < 4; ++s) w2[cv][s] = cadd(w2[cv][s], sl[ww][cv][(4 * s + lr) * 16 + lc]);
        }
        load_v(p - 1, true, false);   // (the next panel's W1 operands: this panel's are used)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int I = w + Q1_NW * h;
            if (I < p + 1 || I >= nti) continue;
#pragma unroll
            for (int cv = 0; cv < 2; ++cv) {
                Cacc U = cacc0();
#pragma unroll
                for (int s = 0; s < 4; ++s) cmma(U, vb[h][s], w2[cv][s]);
                Z[h][cv].r -= U.r;
                Z[h][cv].i -= U.i;
            }
        }
        load_v(p - 1, false, true);
        lds_barrier();   // (LDS only: the next panel's operands stay in flight)
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int cv = 0; cv < 2; ++cv) {
            const int I = w + Q1_NW * h, q = q0 + 16 * cv + lc;
            if (I >= nti) continue;
#pragma unroll
            for (int j4 = 0; j4 < 4; ++j4) {
                const int row = 16 * I + lr + 4 * j4;
                if (q < k && row < d) Vo[(long long)q * d + row] = cget(Z[h][cv], j4);
            }
        }
}

size_t s1_lds(const H2Lay&) { return 0; }   // (static LDS only)
size_t s2_lds(int d) { return 16ull * (size_t)d * ABS; }


}  // namespace

bool heev2_eligible(int d, int kmax) {
    if (!(kmax == d && d >= 32 && d <= H2_MAXD)) return false;
    const H2Lay x = h2lay(d);
    return lds_ok(reinterpret_cast<const void*>(&he2hb_kernel), s1_lds(x)) &&
           lds_ok(reinterpret_cast<const void*>(&hb2st_kernel), s2_lds(d));
}

size_t heev2_extra_bytes(int d, int batch) { return sizeof(double) * (size_t)h2lay(d).stride * batch + 256; }

size_t heev2_request_bytes(int d, int which) {
    const H2Lay x = h2lay(d);
    return which == 0 ? s1_lds(x) : which == 1 ? s2_lds(d) : 0;   // (the back-transform kernels: static LDS only)
}

int launch_heev2(int d, int kmax, int batch, const double* tau, double* scratch, double* V, int* status,
                 const int* active, hipStream_t st, int side_ok) {
    if (!heev2_eligible(d, kmax)) return fail(ACE_ERR_UNSUPPORTED, "two-stage eigensolver: d = %d not supported", d);
    const HeevLayout hl = heev_layout(d, kmax);
    const H2Lay xl = h2lay(d);
    double* xs = scratch + (((size_t)hl.stride * batch + 31) & ~(size_t)31);
    hipLaunchKernelGGL(he2hb_kernel, dim3(batch), dim3(S1_THREADS), s1_lds(xl), st, d, scratch, hl, xs, xl, active);
    hipLaunchKernelGGL(hb2st_kernel, dim3(batch), dim3(S2_THREADS), s2_lds(d), st, d, scratch, hl, xs, xl, active);
    launch_trieig(d, kmax, batch, tau, scratch, status, active, st, side_ok);
    const int groups = (batch + 7) / 8, nc2 = (d + Q2_NV - 1) / Q2_NV, nc1 = (d + Q1_NV - 1) / Q1_NV;
    hipLaunchKernelGGL(bt2q2_kernel, dim3(groups * nc2 * 8), dim3(Q2_THREADS), 0, st, d, kmax, batch, nc2, scratch, hl,
                       xs, xl, V, active);
    hipLaunchKernelGGL(bt2q1_kernel, dim3(groups * nc1 * 8), dim3(Q1_THREADS), 0, st, d, kmax, batch, nc1, scratch, hl,
                       xs, xl, V, active);
    return ACE_OK;
}

}  // namespace ace
