// Private phase-code codebooks (regime P of SURVEY.md §8d: one sensing matrix A_b per
// realisation, as in the per-user loop of Generate_Sensing_Matrix.m) for the r = 1 InferADMM
// iteration (main/src/my_recovery_algorithms/ADMM_v2/inferLowRankV4_multi.m:281-386).
//
// Every A_b of the reference's codebooks is a phase code: after the normalisation of
// inferLowRankV4_multi.m:27-38 each entry is c_b j^k, k in {0, 1, 2, 3}.  The solver's
// per-realisation operators are then
//   A_b, A_b^H   2 bits per entry (64 KiB per realisation at m = 256, n = 1024) instead of
//                4 MiB of complex128,
//   G_b = (I + A_b A_b^H)^{-1}   the Woodbury form of U = inv(A'A + I) (:242/:286-289), Hermitian,
//                stored as its lower triangle in 16 x 16 tiles (544 KiB instead of 16 MiB for U).
// The iteration streams G_b (the HBM-bound part), applies A_b^H on the int8 matrix cores with
// the codebook operand expanded from the 2-bit codes in registers, and keeps every other
// per-realisation vector in LDS.
//
// Setup (per batch, inside the timed region: the reference rebuilds U for every call):
//   pc_pack   phase-code check (every entry exactly c_b j^k) and the 2-bit code images
//   pc_k      K_int = A A^H / c^2 exactly: K_il = sum_k j^(k_ik - k_lk) counted with popcounts
//   pc_gj     G = (I + c^2 K_int)^{-1}: blocked Gauss-Jordan (32-column panels) on HPD I + K
//   pc_tiles  the lower 16 x 16 tiles of G
// Iteration (pgk_kernel, one work-group per realisation), then the one-wave Z-step (wmode):
//   T = (Y - M/mu) - A V           A V = AX of the previous Y-step when V is that iteration's X
//                                  (RealState::avok), else the digit-plane product A V
//   g = G T                        Hermitian tiles: each off-diagonal tile serves G T and G^H T
//   Y-step                         ArgMinY, M update (:326-337), sums, opt_Y
//   W = A^H g, |A^H Y|^2, |A^H (Y - Y0)|^2   one int8 GEMM with three digit-plane right-hand sides
#include "ace_i8.hpp"

#include <algorithm>
#include <cstdlib>

namespace ace {

namespace {

constexpr int PNT = 256;   // threads of the per-realisation kernels

// Phase timestamps of work-group 5 (diagnostic build only: -DACE_PHASE_STAMPS)
#ifdef ACE_PHASE_STAMPS
#define PSTAMP_DECL unsigned long long ts_[12] = {}
#define PSTAMP(i) do { if (blockIdx.x == 5 && threadIdx.x == 0) ts_[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define PSTAMP_PRINT(name, k) do { if (blockIdx.x == 5 && threadIdx.x == 0) { printf("%s", name); for (int i_ = 1; i_ < k; ++i_) printf(" %llu", ts_[i_] - ts_[i_ - 1]); printf("\n"); } } while (0)
#else
#define PSTAMP_DECL
#define PSTAMP(i)
#define PSTAMP_PRINT(name, k)
#endif

struct PcDims {
    int m, n, mt, mp, mp32, nb32, ntile, nctH, nksH, nkgH, nctA, nksA, nkgA, nwR;
};
__host__ __device__ __forceinline__ PcDims pc_dims(int m, int n) {
    PcDims d;
    d.m = m;
    d.n = n;
    d.mt = (m + 15) >> 4;          // 16-row tiles of G (and 16-complex K-steps of A^H)
    d.mp = 16 * d.mt;
    d.mp32 = 32 * ((m + 31) >> 5); // Gauss-Jordan panel granularity
    d.nb32 = d.mp32 >> 5;
    d.ntile = d.mt * (d.mt + 1) / 2;
    d.nctH = (n + 15) >> 4;        // A^H: 16 output complex per 32-column MFMA tile
    d.nksH = d.mt;                 //      16 input complex per K-step
    d.nkgH = (d.nksH + 7) >> 3;    //      8 K-steps per 16-byte code load
    d.nctA = d.mt;                 // A:   outputs over m
    d.nksA = (n + 15) >> 4;        //      inputs over n
    d.nkgA = (d.nksA + 7) >> 3;
    d.nwR = (n + 15) >> 4;         // row-major code dwords per row (16 codes each)
    return d;
}
__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
    return __builtin_amdgcn_perm(s0, s1, sel);
}

// Code image layout of one realisation (uint4 = one lane's 8 K-steps): for output tile ct,
// K-step group kg, local output o (0..15), input half h (0, 1):
//   uint4 ((ct * nkg + kg) * 16 + o) * 2 + h;  dword j covers K-steps 8 kg + 2 j + p (p = 0, 1);
//   the code of input u (0..7, input 16 ks + 8 h + u) sits at bit 8 (u & 3) + 2 (2 p + (u >> 2)),
// so that (dword >> (4 p)) & 0x03030303 and (dword >> (4 p + 2)) & 0x03030303 hold the codes of
// inputs 0..3 and 4..7 one per byte: the selectors of the v_perm lookups below.
__device__ __forceinline__ int code_shift(int p, int u) { return 8 * (u & 3) + 2 * (2 * p + (u >> 2)); }

// ---- setup -------------------------------------------------------------------------------

// One work-group per (realisation, 32-row block of A_b): check and encode the rows (c_b = the
// first entry's magnitude; any entry that is not exactly c_b j^k sets *flag), then emit
// the A^H image (this block is one K-step pair), the A image (two output tiles) and the
// row-major codes (16 per dword) used by pc_k.
__global__ __launch_bounds__(PNT) void pc_pack_kernel(int m, int n, const double* __restrict__ A,
                                                      double* __restrict__ cb, uint32_t* __restrict__ cH,
                                                      uint32_t* __restrict__ cA, uint32_t* __restrict__ cR,
                                                      int* __restrict__ flag) {
    extern __shared__ unsigned char cs[];   // [32][np] code bytes (0 outside A)
    const PcDims d = pc_dims(m, n);
    const int b = blockIdx.x, rb = blockIdx.y, t = threadIdx.x;
    const int np = 16 * d.nksA;
    const d2* a = reinterpret_cast<const d2*>(A) + (long long)b * m * n;
    // c_b from the first entry; every entry must then be exactly c_b j^k
    const d2 a00 = a[0];
    const double c = fmax(fabs(a00.x), fabs(a00.y));
    int bad = !(c > 0.0 && c <= 1.7e308);
    if (rb == 0 && t == 0) cb[b] = c;
    for (int e = t; e < 32 * np; e += PNT) {
        const int il = e / np, k = e - il * np, i = 32 * rb + il;
        unsigned char code = 0;
        if (i < m && k < n) {
            const d2 v = a[(long long)i * n + k];
            if (v.y == 0.0 && v.x == c) code = 0;
            else if (v.x == 0.0 && v.y == c) code = 1;
            else if (v.y == 0.0 && v.x == -c) code = 2;
            else if (v.x == 0.0 && v.y == -c) code = 3;
            else bad = 1;
        }
        cs[e] = code;
    }
    if (bad) atomicOr(flag, 1);
    __syncthreads();
    auto code_at = [&](int il, int k) -> uint32_t { return cs[il * np + k]; };
    // A^H image: output k (tiles of 16), inputs i = rows of this block (K-steps 2 rb, 2 rb + 1)
    {
        const int ks0 = 2 * rb, kg = ks0 >> 3, j = (ks0 & 7) >> 1;
        uint32_t* base = cH + (size_t)b * d.nctH * d.nkgH * 128;
        for (int e = t; e < d.nctH * 32; e += PNT) {
            const int ct = e >> 5, o = (e >> 1) & 15, h = e & 1, kc = 16 * ct + o;
            uint32_t w = 0;
            if (kc < n)
#pragma unroll
                for (int p = 0; p < 2; ++p)
#pragma unroll
                    for (int u = 0; u < 8; ++u) w |= code_at(16 * p + 8 * h + u, kc) << code_shift(p, u);
            base[((((size_t)ct * d.nkgH + kg) * 16 + o) * 2 + h) * 4 + j] = w;
        }
    }
    // A image: outputs i (tiles 2 rb, 2 rb + 1), inputs k over n
    {
        uint32_t* base = cA + (size_t)b * d.nctA * d.nkgA * 128;
        for (int e = t; e < 2 * d.nkgA * 128; e += PNT) {
            const int tl = e / (d.nkgA * 128), r = e - tl * d.nkgA * 128;
            const int kg = r >> 7, o = (r >> 3) & 15, h = (r >> 2) & 1, j = r & 3;
            const int ct = 2 * rb + tl;
            if (ct >= d.nctA) continue;
            uint32_t w = 0;
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const int ks = 8 * kg + 2 * j + p;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int k = 16 * ks + 8 * h + u;
                    if (k < np) w |= code_at(16 * tl + o, k) << code_shift(p, u);
                }
            }
            base[((((size_t)ct * d.nkgA + kg) * 16 + o) * 2 + h) * 4 + j] = w;
        }
    }
    // row-major codes
    for (int e = t; e < 32 * d.nwR; e += PNT) {
        const int il = e / d.nwR, wd = e - il * d.nwR, i = 32 * rb + il;
        if (i >= m) continue;
        uint32_t w = 0;
#pragma unroll
        for (int u = 0; u < 16; ++u) w |= code_at(il, 16 * wd + u) << (2 * u);
        cR[((size_t)b * m + i) * d.nwR + wd] = w;
    }
}

// I + K for one 32 x 32 block pair (I, L) of realisation b, L <= I:
//   K_il = sum_k a_ik conj(a_lk) = c^2 sum_k j^(k_ik - k_lk) = c^2 ((n0 - n2) + j (n1 - n3))
// with n_d the number of k with (k_ik - k_lk) mod 4 = d (2-bit SWAR difference, popcounts).
// Written to both triangles of Gw (row-major, mp32 x mp32, identity outside m).
__global__ __launch_bounds__(PNT) void pc_k_kernel(int m, int n, const uint32_t* __restrict__ cR,
                                                   const double* __restrict__ cb, double* __restrict__ Gw) {
    const PcDims d = pc_dims(m, n);
    const int b = blockIdx.x, p = blockIdx.y, t = threadIdx.x;
    int I = (int)((sqrt(8.0 * p + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= p) ++I;
    while (I * (I + 1) / 2 > p) --I;
    const int L = p - I * (I + 1) / 2;
    extern __shared__ uint32_t rows[];   // [2][32][nwR + 1]
    const int rs = d.nwR + 1;
    const uint32_t* src = cR + (size_t)b * m * d.nwR;
    for (int e = t; e < 64 * d.nwR; e += PNT) {
        const int r = e / d.nwR, wd = e - r * d.nwR, blk = r >> 5, il = r & 31;
        const int i = 32 * (blk ? L : I) + il;
        rows[r * rs + wd] = i < m ? src[(size_t)i * d.nwR + wd] : 0u;
    }
    __syncthreads();
    const int i2 = t >> 4, l2 = t & 15;
    int c1[2][2] = {}, c2[2][2] = {}, c3[2][2] = {};
    const uint32_t* ra = rows + (2 * i2) * rs;
    const uint32_t* rl = rows + (32 + 2 * l2) * rs;
    constexpr uint32_t L55 = 0x55555555u;
    for (int wd = 0; wd < d.nwR; ++wd) {
        const uint32_t a0 = ra[wd], a1 = ra[rs + wd], b0 = rl[wd], b1 = rl[rs + wd];
        const uint32_t av[2] = {a0, a1}, bv[2] = {b0, b1};
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) {
                const uint32_t aa = av[x], bb = bv[y];
                const uint32_t xo = aa ^ bb;
                const uint32_t lo = xo & L55;                           // d bit 0
                const uint32_t hi = ((xo >> 1) ^ (~aa & bb)) & L55;     // d bit 1 (with the borrow)
                c1[x][y] += __builtin_popcount(lo & ~hi);
                c2[x][y] += __builtin_popcount(hi & ~lo);
                c3[x][y] += __builtin_popcount(lo & hi);
            }
    }
    const double c = cb[b], c2v = c * c;
    d2* G = reinterpret_cast<d2*>(Gw) + (size_t)b * d.mp32 * d.mp32;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            const int i = 32 * I + 2 * i2 + x, l = 32 * L + 2 * l2 + y;
            d2 v = make_double2(i == l ? 1.0 : 0.0, 0.0);
            if (i < m && l < m) {
                const int n0 = n - c1[x][y] - c2[x][y] - c3[x][y];
                v.x += c2v * (double)(n0 - c2[x][y]);
                v.y = c2v * (double)(c1[x][y] - c3[x][y]);
            }
            G[(size_t)i * d.mp32 + l] = v;
            G[(size_t)l * d.mp32 + i] = make_double2(v.x, -v.y);
        }
}

// ---- blocked Gauss-Jordan inversion of the HPD I + K (no pivoting), 32-column panels.
// Step k:  P = A_kk^{-1};  row panel A_kj <- P A_kj (j != k), A_kk <- P          (gj_panel)
//          A_ij <- A_ij - A_ik A_kj,  A_ik <- -A_ik P      for i != k            (gj_update)
constexpr int GJS = 33;   // LDS row stride of a 32 x 32 block (complex)
__global__ __launch_bounds__(PNT) void gj_panel_kernel(int mp32, int k, double* __restrict__ Gw) {
    __shared__ d2 Ps[32 * GJS];
    __shared__ d2 rowb[32], colb[32];
    const int t = threadIdx.x;
    d2* G = reinterpret_cast<d2*>(Gw) + (size_t)blockIdx.x * mp32 * mp32;
    const size_t k0 = 32 * (size_t)k;
    for (int e = t; e < 1024; e += PNT) Ps[(e >> 5) * GJS + (e & 31)] = G[(k0 + (e >> 5)) * mp32 + k0 + (e & 31)];
    __syncthreads();
    for (int p = 0; p < 32; ++p) {
        if (t < 32) {
            const d2 pv = Ps[p * GJS + p];
            const double den = pv.x * pv.x + pv.y * pv.y;
            const d2 pinv = make_double2(pv.x / den, -pv.y / den);
            const d2 a = (t == p) ? make_double2(1.0, 0.0) : Ps[p * GJS + t];
            rowb[t] = cmul(a, pinv);
            colb[t] = Ps[t * GJS + p];
        }
        __syncthreads();
        for (int e = t; e < 1024; e += PNT) {
            const int r = e >> 5, c = e & 31;
            if (r == p) {
                Ps[r * GJS + c] = rowb[c];
            } else {
                const d2 base = (c == p) ? make_double2(0.0, 0.0) : Ps[r * GJS + c];
                Ps[r * GJS + c] = csub(base, cmul(colb[r], rowb[c]));
            }
        }
        __syncthreads();
    }
    // row panel: column j of P A_k*, one thread per column
    for (int j = t; j < mp32; j += PNT) {
        if ((size_t)j >= k0 && (size_t)j < k0 + 32) {
            for (int r = 0; r < 32; ++r) G[(k0 + r) * mp32 + j] = Ps[r * GJS + (j - (int)k0)];
            continue;
        }
        d2 col[32];
#pragma unroll
        for (int c = 0; c < 32; ++c) col[c] = G[(k0 + c) * mp32 + j];
        for (int r0 = 0; r0 < 32; r0 += 4) {   // four rows: independent FMA chains
            double sr[4] = {0.0, 0.0, 0.0, 0.0}, si[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int c = 0; c < 32; ++c)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const d2 pv = Ps[(r0 + u) * GJS + c];
                    sr[u] = fma(pv.x, col[c].x, fma(-pv.y, col[c].y, sr[u]));
                    si[u] = fma(pv.x, col[c].y, fma(pv.y, col[c].x, si[u]));
                }
#pragma unroll
            for (int u = 0; u < 4; ++u) G[(k0 + r0 + u) * mp32 + j] = make_double2(sr[u], si[u]);
        }
    }
}

__global__ __launch_bounds__(PNT) void gj_update_kernel(int mp32, int k, double* __restrict__ Gw) {
    __shared__ d2 Cs[32 * GJS], Pm[32 * GJS];
    const int t = threadIdx.x;
    const int I = (int)blockIdx.y < k ? (int)blockIdx.y : (int)blockIdx.y + 1;
    d2* G = reinterpret_cast<d2*>(Gw) + (size_t)blockIdx.x * mp32 * mp32;
    const size_t k0 = 32 * (size_t)k, i0 = 32 * (size_t)I;
    for (int e = t; e < 1024; e += PNT) {
        const int r = e >> 5, c = e & 31;
        Cs[r * GJS + c] = G[(i0 + r) * mp32 + k0 + c];
        Pm[r * GJS + c] = G[(k0 + r) * mp32 + k0 + c];
    }
    __syncthreads();
    for (int j = t; j < mp32; j += PNT) {
        const bool inblk = (size_t)j >= k0 && (size_t)j < k0 + 32;
        d2 rc[32];
#pragma unroll
        for (int c = 0; c < 32; ++c) rc[c] = inblk ? Pm[c * GJS + (j - (int)k0)] : G[(k0 + c) * mp32 + j];
        for (int r0 = 0; r0 < 32; r0 += 4) {   // four rows: independent FMA chains
            d2 o[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) o[u] = inblk ? make_double2(0.0, 0.0) : G[(i0 + r0 + u) * mp32 + j];
            double sr[4] = {0.0, 0.0, 0.0, 0.0}, si[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int c = 0; c < 32; ++c)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const d2 cv = Cs[(r0 + u) * GJS + c];
                    sr[u] = fma(cv.x, rc[c].x, fma(-cv.y, rc[c].y, sr[u]));
                    si[u] = fma(cv.x, rc[c].y, fma(cv.y, rc[c].x, si[u]));
                }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                G[(i0 + r0 + u) * mp32 + j] = make_double2(o[u].x - sr[u], o[u].y - si[u]);
        }
    }
}

// ---- recursive block inversion of the HPD I + K (Schur complements; the default since r02).
// For H = [[A, B^H], [B, D]] (A: h x h, D: r x r):
//   F = B A^{-1},  S = D - F B^H,  T = F^H S^{-1},
//   H^{-1} = [[A^{-1} + T F, -T], [-T^H, S^{-1}]]
// with A^{-1} and S^{-1} by recursion down to 32 x 32 blocks (inv32_kernel, Gauss-Jordan in LDS).
// Every product is one batched launch of the complex 3M GEMM (ace_gemm.hip) over the batch's
// matrices: 2/3 m^3 complex MACs per matrix against m^3 for the full Gauss-Jordan, on the matrix
// cores instead of LDS-broadcast FMAs.  S is HPD whenever H is, so no pivoting is needed.

// in-place inverse of one HPD 32 x 32 block per realisation (Gauss-Jordan without pivoting)
__global__ __launch_bounds__(PNT) void inv32_kernel(int ld, long long stride, double* __restrict__ H) {
    __shared__ d2 Ps[32 * GJS];
    __shared__ d2 rowb[32], colb[32];
    const int t = threadIdx.x;
    d2* G = reinterpret_cast<d2*>(H) + (size_t)blockIdx.x * stride;
    for (int e = t; e < 1024; e += PNT) Ps[(e >> 5) * GJS + (e & 31)] = G[(size_t)(e >> 5) * ld + (e & 31)];
    __syncthreads();
    for (int p = 0; p < 32; ++p) {
        if (t < 32) {
            const d2 pv = Ps[p * GJS + p];
            const double den = pv.x * pv.x + pv.y * pv.y;
            const d2 pinv = make_double2(pv.x / den, -pv.y / den);
            const d2 a = (t == p) ? make_double2(1.0, 0.0) : Ps[p * GJS + t];
            rowb[t] = cmul(a, pinv);
            colb[t] = Ps[t * GJS + p];
        }
        __syncthreads();
        for (int e = t; e < 1024; e += PNT) {
            const int r = e >> 5, c = e & 31;
            if (r == p) {
                Ps[r * GJS + c] = rowb[c];
            } else {
                const d2 base = (c == p) ? make_double2(0.0, 0.0) : Ps[r * GJS + c];
                Ps[r * GJS + c] = csub(base, cmul(colb[r], rowb[c]));
            }
        }
        __syncthreads();
    }
    for (int e = t; e < 1024; e += PNT) G[(size_t)(e >> 5) * ld + (e & 31)] = Ps[(e >> 5) * GJS + (e & 31)];
}

// F (rows x cols, ld cols) -> Fh = F^H (cols x rows, ld rows)                       (neg = false)
// T (rows x cols, ld cols) -> Up = -T (ldu), Lo = -T^H (ldl)                         (neg = true)
template <bool NEG>
__global__ __launch_bounds__(PNT) void ctrans_kernel(int rows, int cols, const double* __restrict__ src,
                                                     long long sstride, double* __restrict__ up, int ldu,
                                                     double* __restrict__ lo, int ldl, long long dstride) {
    __shared__ d2 tile[32][33];
    const int b = blockIdx.z, tr = blockIdx.y, tc = blockIdx.x, t = threadIdx.x;
    const d2* s = reinterpret_cast<const d2*>(src) + (size_t)b * sstride;
    d2* u = reinterpret_cast<d2*>(up) + (size_t)b * dstride;
    d2* l = reinterpret_cast<d2*>(lo) + (size_t)b * dstride;
    for (int e = t; e < 1024; e += PNT) {
        const int r = e >> 5, c = e & 31, i = 32 * tr + r, j = 32 * tc + c;
        d2 v = make_double2(0.0, 0.0);
        if (i < rows && j < cols) v = s[(size_t)i * cols + j];
        if (NEG) {
            v = make_double2(-v.x, -v.y);
            if (i < rows && j < cols) u[(size_t)i * ldu + j] = v;
        }
        tile[r][c] = v;
    }
    __syncthreads();
    for (int e = t; e < 1024; e += PNT) {
        const int r = e >> 5, c = e & 31, j = 32 * tc + r, i = 32 * tr + c;   // out (j, i) = conj(in (i, j))
        if (i < rows && j < cols) {
            const d2 v = tile[c][r];
            l[(size_t)j * ldl + i] = make_double2(v.x, -v.y);
        }
    }
}

// lower 16 x 16 tiles of G, column-major inside a tile: Gt[b][I (I + 1) / 2 + K][c][r] = G[16 I + r][16 K + c]
__global__ __launch_bounds__(PNT) void pc_tiles_kernel(int m, const double* __restrict__ Gw, double* __restrict__ Gt) {
    const PcDims d = pc_dims(m, 16);
    const int b = blockIdx.x, idx = blockIdx.y, t = threadIdx.x;
    int I = (int)((sqrt(8.0 * idx + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= idx) ++I;
    while (I * (I + 1) / 2 > idx) --I;
    const int K = idx - I * (I + 1) / 2;
    const int r = t >> 4, c = t & 15, i = 16 * I + r, k = 16 * K + c;
    const d2* G = reinterpret_cast<const d2*>(Gw) + (size_t)b * d.mp32 * d.mp32;
    const d2 v = (i < m && k < m) ? G[(size_t)i * d.mp32 + k] : make_double2(0.0, 0.0);
    reinterpret_cast<d2*>(Gt)[((size_t)b * d.ntile + idx) * 256 + c * 16 + r] = v;
}

// ---- the iteration kernel ----------------------------------------------------------------

// Codebook operand of one K-step from the lane's code dword (8 inputs, byte order
// x0..x3 y0..y3 x4..x7 y4..y7 of the K half): lutX / lutY map a code to the int8 entry that
// multiplies the input's real / imaginary part for this lane's output real.
__device__ __forceinline__ i4v code_frag(uint32_t dw, int p, uint32_t lutX, uint32_t lutY) {
    const uint32_t s0 = (dw >> (4 * p)) & 0x03030303u, s1 = (dw >> (4 * p + 2)) & 0x03030303u;
    // the table in both source operands: selectors 0..3 and 4..7 read the same bytes
    return i4v{(int)perm(lutX, lutX, s0), (int)perm(lutY, lutY, s0), (int)perm(lutX, lutX, s1), (int)perm(lutY, lutY, s1)};
}
// entries as int8 bytes indexed by the code k (entry c j^k = c (p + j q)):
//   P = Re j^k = [1, 0, -1, 0],  Q = Im j^k = [0, 1, 0, -1]
constexpr uint32_t LUT_P = 0x00FF0001u, LUT_Q = 0xFF000100u, LUT_NQ = 0x0100FF00u;


// digits of 4 consecutive inputs i0..i0+3 (i0 % 4 == 0) of one right-hand side into its 8 LDS rows:
// row(tt) is the byte offset of digit tt's row; the K-step byte slots follow the code layout
// (x0..x3 y0..y3 x4..x7 y4..y7 per 16-byte half of a 16-input K-step)
template <class RowOff>
__device__ __forceinline__ void put_digits4(int8_t* Ad, RowOff row, int i0, const d2 (&v)[4], double p2) {
    uint32_t dx[4][8], dy[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        digits1(v[u].x * p2, dx[u]);
        digits1(v[u].y * p2, dy[u]);
    }
    const int off = 32 * (i0 >> 4) + 16 * ((i0 >> 3) & 1) + 8 * ((i0 >> 2) & 1);
#pragma unroll
    for (int tt = 0; tt < 8; ++tt) {
        const uint32_t xw = dx[0][tt] | (dx[1][tt] << 8) | (dx[2][tt] << 16) | (dx[3][tt] << 24);
        const uint32_t yw = dy[0][tt] | (dy[1][tt] << 8) | (dy[2][tt] << 16) | (dy[3][tt] << 24);
        *reinterpret_cast<uint32_t*>(Ad + row(tt) + off) = xw;
        *reinterpret_cast<uint32_t*>(Ad + row(tt) + off + 4) = yw;
    }
}

__device__ __forceinline__ d2 d2zero() { return make_double2(0.0, 0.0); }

// owner wave of 16-row tile row I of G (snake over groups of 4 rows: balanced triangle)
__device__ __forceinline__ int tile_owner(int I) {
    const int g = I >> 2, r = I & 3;
    return (g & 1) ? 3 - r : r;
}

// LDS carve of pgk_kernel (bytes), shared by the kernel and the launcher
struct PgkLds {
    int ts, grow, cp, list, ad, total, rstH, rstA;
};
__host__ __device__ __forceinline__ PgkLds pgk_lds(int m, int n) {
    const PcDims d = pc_dims(m, n);
    PgkLds L;
    L.rstH = 32 * d.nksH + 16;    // A^H digit rows: 4 right-hand sides x 8 digits
    L.rstA = 32 * d.nksA + 16;    // A digit rows (cold A V): 8 digits of V
    const int adb = 32 * L.rstH > 8 * L.rstA ? 32 * L.rstH : 8 * L.rstA;
    L.ts = 0;                                  // d2 [mp]: T, then g
    L.grow = L.ts + 16 * d.mp;                 // d2 [mp]: row sums of G T, then Y_new (and A V reals)
    L.cp = L.grow + 16 * d.mp;                 // d2 [4][mp]: per-wave column sums, then dY in cp[0]
    L.list = L.cp + 4 * 16 * d.mp;             // uint16 [4][64]: each wave's tile stream
    L.ad = (L.list + 4 * 64 * 2 + 15) & ~15;   // digit planes
    L.total = L.ad + adb;
    return L;
}

// avs[0 .. 2m) = c A v for one realisation on the int8 matrix cores (all PNT threads): the 8
// digit planes of v (vget(k), k < n, against 2^e >= bound) in 8 LDS rows of rstA bytes (MFMA rows
// lds_row(0, tt) = 8 (tt >> 2) + (tt & 3); the other 24 rows read as zero), the codebook operand
// expanded from the realisation's A image cA.  Ends with the block synchronised.
template <class VGet>
__device__ __forceinline__ void pc_av_block(const PcDims& d, int rstA, int8_t* Ad, const uint4* __restrict__ cA,
                                            double bound, double c, VGet vget, double* avs) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    double p2, sc;
    plane_scale(bound, c, p2, sc);
    for (int g4 = t; g4 < 4 * d.nksA; g4 += PNT) {
        d2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = 4 * g4 + u;
            v[u] = k < d.n ? vget(k) : make_double2(0.0, 0.0);
        }
        put_digits4(Ad, [&](int tt) { return tt * rstA; }, 4 * g4, v, p2);
    }
    __syncthreads();
    const int r32 = lane & 31;
    const bool rok = (r32 & 4) == 0 && r32 < 16;
    const int8_t* abase = Ad + ((r32 & 3) + 4 * (r32 >> 3)) * rstA + 16 * (lane >> 5);
    const bool im = lane & 1;   // output real: even = Re, odd = Im
    const uint32_t lutX = im ? LUT_Q : LUT_P, lutY = im ? LUT_P : LUT_NQ;   // a v: (p x - q y, q x + p y)
    for (int ct = w; ct < d.nctA; ct += PNT / 64) {
        const uint4* cp = cA + (size_t)ct * d.nkgA * 32 + ((lane & 31) >> 1) * 2 + (lane >> 5);
        i16v acc = i16v{};
        for (int kg = 0; kg < d.nkgA; ++kg) {
            const uint4 cw = cp[(size_t)kg * 32];
            const uint32_t cwv[4] = {cw.x, cw.y, cw.z, cw.w};
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    const int ks = 8 * kg + 2 * j + p;
                    if (ks < d.nksA) {
                        const i4v af = rok ? *reinterpret_cast<const i4v*>(abase + 32 * ks) : i4v{0, 0, 0, 0};
                        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(af, code_frag(cwv[j], p, lutX, lutY), acc, 0, 0, 0);
                    }
                }
        }
        const int col = 32 * ct + (lane & 31);
        if (lane < 32 && col < 2 * d.m) avs[col] = sc * recombine(acc, 0);
    }
    __syncthreads();
}

// init (:296-300): P0 = A X0 for the private phase-code path (one work-group per realisation)
__global__ __launch_bounds__(PNT) void pc_apply_a_kernel(int m, int n, const uint32_t* __restrict__ codesA,
                                                         const double* __restrict__ cb, const double* __restrict__ X0,
                                                         double* __restrict__ P0) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ double red[2][PNT / 64];
    const PcDims d = pc_dims(m, n);
    const int b = blockIdx.x, t = threadIdx.x;
    const d2* x = reinterpret_cast<const d2*>(X0) + (long long)b * n;
    VMax vm;
    for (int k = t; k < n; k += PNT) vm.add(x[k]);
    const double mx = wave_max(vm.m), sn = wave_sum(vm.s);
    if ((t & 63) == 0) {
        red[0][t >> 6] = mx;
        red[1][t >> 6] = sn;
    }
    __syncthreads();
    double bound = 0.0, sticky = 0.0;
    for (int w = 0; w < PNT / 64; ++w) {
        bound = fmax(bound, red[0][w]);
        sticky += red[1][w];
    }
    double* avs = reinterpret_cast<double*>(smem);
    int8_t* Ad = reinterpret_cast<int8_t*>(smem) + ((16 * d.mp + 15) & ~15);
    pc_av_block(d, 32 * d.nksA + 16, Ad, reinterpret_cast<const uint4*>(codesA) + (size_t)b * d.nctA * d.nkgA * 32,
                bound + sticky, cb[b], [&](int k) { return x[k]; }, avs);
    for (int e = t; e < 2 * m; e += PNT) P0[(long long)b * 2 * m + e] = avs[e];
}

__global__ __launch_bounds__(PNT) void pgk_kernel(PgkArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ double red[4][12];
    const int m = a.m, n = a.n, b = blockIdx.x;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    RealState* rs = a.rs + b;
    if (rs->done) return;
    PSTAMP_DECL;
    PSTAMP(0);
    const PcDims d = pc_dims(m, n);
    const PgkLds L = pgk_lds(m, n);
    d2* Ts = reinterpret_cast<d2*>(smem + L.ts);
    d2* grow = reinterpret_cast<d2*>(smem + L.grow);
    d2* cp = reinterpret_cast<d2*>(smem + L.cp);
    uint16_t* tl = reinterpret_cast<uint16_t*>(smem + L.list);
    int8_t* Ad = reinterpret_cast<int8_t*>(smem + L.ad);
    const double mu = rs->mu, imu = 1.0 / mu, c = a.cb[b];
    const int avok = a.AX && rs->avok, oys = rs->optysrc;
    const long long om = (long long)b * m;
    const int i = t;
    const bool iv = i < m;
    d2 yo = d2zero(), mi = d2zero();
    double bi = 0.0;
    if (iv) {
        yo = reinterpret_cast<const d2*>(a.Yo)[om + i];
        mi = reinterpret_cast<const d2*>(a.M)[om + i];
        bi = a.B[om + i];
        // deferred opt_Y (RealState::optysrc): the best Y_new is in the buffer this Y-step overwrites
        if (a.yn_id && oys == a.yn_id) reinterpret_cast<d2*>(a.optY)[om + i] = reinterpret_cast<const d2*>(a.Yn)[om + i];
    }
    for (int e = t; e < 4 * d.mp; e += PNT) cp[e] = d2zero();
    // this wave's stream of G tiles: owned tile rows ascending, K = 0..I
    int ntw = 0;
    for (int I = 0; I < d.mt; ++I)
        if (tile_owner(I) == w) {
            if (lane <= I) tl[64 * w + ntw + lane] = (uint16_t)((I << 8) | lane);
            ntw += I + 1;
        }
    ntw = __builtin_amdgcn_readfirstlane(ntw);
    // the first G tiles are requested now: their latency overlaps the T phase
    const int r16 = lane & 15, q4 = lane >> 4;
    const d2* gtb = reinterpret_cast<const d2*>(a.Gt) + (size_t)b * d.ntile * 256 + (4 * q4) * 16 + r16;
    auto tptr = [&](int f) -> const d2* {
        const int code = tl[64 * w + (f < ntw ? f : (ntw > 0 ? ntw - 1 : 0))];
        const int I = code >> 8, K = code & 255;
        return gtb + (size_t)(I * (I + 1) / 2 + K) * 256;
    };
    auto load = [&](d2 (&gv)[4], int f) {
        const d2* p = tptr(f);
#pragma unroll
        for (int j = 0; j < 4; ++j) {   // streamed once per iteration: non-temporal (keep L2 for the rest)
            typedef double dv2 __attribute__((ext_vector_type(2)));
            const dv2 v = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(p + 16 * j));
            gv[j] = make_double2(v.x, v.y);
        }
    };
    d2 b0[4], b1[4], b2[4], b3[4];
    if (ntw > 0) {   // (a wave owns no tile row when m <= 48)
        load(b0, 0);
        load(b1, 1);
        load(b2, 2);
    }

    // ---- T = (Y - M/mu) - A V  (the expression of i8a_block / gyk_kernel)
    if (avok) {
        if (iv) {
            const d2 ax = reinterpret_cast<const d2*>(a.AX)[om + i];
            Ts[i] = make_double2(fma(-mi.x, imu, yo.x) - ax.x, fma(-mi.y, imu, yo.y) - ax.y);
        } else if (i < d.mp) {
            Ts[i] = d2zero();
        }
    } else {
        const d2* zp = reinterpret_cast<const d2*>(a.Z) + (long long)b * n;
        const d2* np = rs->nzero ? reinterpret_cast<const d2*>(a.zeros) : reinterpret_cast<const d2*>(a.N) + (long long)b * n;
        double* avs = reinterpret_cast<double*>(grow);
        pc_av_block(d, L.rstA, Ad, reinterpret_cast<const uint4*>(a.codesA) + (size_t)b * d.nctA * d.nkgA * 32,
                    rs->vbound, c, [&](int k) {
                        const d2 z = zp[k], nn = np[k];
                        return make_double2(fma(-nn.x, imu, z.x), fma(-nn.y, imu, z.y));
                    }, avs);
        __syncthreads();
        if (iv) Ts[i] = make_double2(fma(-mi.x, imu, yo.x) - avs[2 * i], fma(-mi.y, imu, yo.y) - avs[2 * i + 1]);
        else if (i < d.mp) Ts[i] = d2zero();
    }
    __syncthreads();
    PSTAMP(1);

    // ---- g = G T over the lower tiles: a tile (I, K) adds G_IK T_K to rows I (lane-owned row
    // sums) and, for K < I, G_IK^H T_I to rows K (reduced over the tile's 16 rows, accumulated in
    // the wave's column sums).  Each wave streams its tile rows with loads three tiles ahead.
    {
        const int q = q4;
        d2 racc = d2zero(), trow = d2zero();
        d2* cpw = cp + w * d.mp;
        auto compute = [&](const d2 (&gv)[4], int f) {
            const int code = tl[64 * w + f];
            const int I = code >> 8, K = code & 255;
            if (K == 0) {
                racc = d2zero();
                trow = Ts[16 * I + r16];
            }
            d2 v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const d2 tv = Ts[16 * K + 4 * q + j], gg = gv[j];
                racc.x = fma(gg.x, tv.x, fma(-gg.y, tv.y, racc.x));
                racc.y = fma(gg.x, tv.y, fma(gg.y, tv.x, racc.y));
                v[j] = make_double2(fma(gg.x, trow.x, gg.y * trow.y), fma(gg.x, trow.y, -gg.y * trow.x));   // conj(g) t
            }
            if (K < I) {   // reduce-scatter of v[0..3] over the 16 rows of the tile
                const bool s8 = r16 & 8, s4 = r16 & 4;
                const d2 k0 = s8 ? v[2] : v[0], k1 = s8 ? v[3] : v[1], o0 = s8 ? v[0] : v[2], o1 = s8 ? v[1] : v[3];
                d2 u0, u1;
                u0.x = k0.x + __shfl_xor(o0.x, 8, 64);
                u0.y = k0.y + __shfl_xor(o0.y, 8, 64);
                u1.x = k1.x + __shfl_xor(o1.x, 8, 64);
                u1.y = k1.y + __shfl_xor(o1.y, 8, 64);
                const d2 kk = s4 ? u1 : u0, oo = s4 ? u0 : u1;
                d2 x;
                x.x = kk.x + __shfl_xor(oo.x, 4, 64);
                x.y = kk.y + __shfl_xor(oo.y, 4, 64);
                x.x += __shfl_xor(x.x, 2, 64);
                x.y += __shfl_xor(x.y, 2, 64);
                x.x += __shfl_xor(x.x, 1, 64);
                x.y += __shfl_xor(x.y, 1, 64);
                if ((r16 & 3) == 0) {
                    const int col = 16 * K + 4 * q + 2 * (s8 ? 1 : 0) + (s4 ? 1 : 0);
                    const d2 o = cpw[col];
                    cpw[col] = make_double2(o.x + x.x, o.y + x.y);
                }
            }
            if (K == I) {   // end of the tile row: sum the four column quarters
                racc.x += __shfl_xor(racc.x, 16, 64);
                racc.y += __shfl_xor(racc.y, 16, 64);
                racc.x = xor32_sum(racc.x);
                racc.y = xor32_sum(racc.y);
                if (q == 0) grow[16 * I + r16] = racc;
            }
        };
        for (int f0 = 0; f0 < ntw; f0 += 4) {
            load(b3, f0 + 3);
            compute(b0, f0);
            load(b0, f0 + 4);
            if (f0 + 1 < ntw) compute(b1, f0 + 1);
            load(b1, f0 + 5);
            if (f0 + 2 < ntw) compute(b2, f0 + 2);
            load(b2, f0 + 6);
            if (f0 + 3 < ntw) compute(b3, f0 + 3);
        }
    }
    __syncthreads();
    PSTAMP(2);

    // A^H codes of this wave's first two output tiles, requested before the Y-step
    const uint4* cpH = reinterpret_cast<const uint4*>(a.codesH) + (size_t)b * d.nctH * d.nkgH * 32 +
                       ((lane & 31) >> 1) * 2 + (lane >> 5);
    auto cload = [&](uint4 (&cw)[2], int ct) {
        const int cc = ct < d.nctH ? ct : d.nctH - 1;
#pragma unroll
        for (int kg = 0; kg < 2; ++kg) cw[kg] = kg < d.nkgH ? cpH[((size_t)cc * d.nkgH + kg) * 32] : make_uint4(0, 0, 0, 0);
    };
    uint4 cq0[2], cq1[2], cq2[2];
    cload(cq0, w);
    cload(cq1, w + 4);

    // ---- Y-step on entry i (gyk_kernel's arithmetic): g, ArgMinY, M update, sums
    d2 gv = d2zero(), y = d2zero(), dy = d2zero();
    double sv[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};   // 5 sums, 3 max |.|, 3 NaN-sticky terms
    if (iv) {
        gv = grow[i];
#pragma unroll
        for (int q = 0; q < 4; ++q) gv = cadd(gv, cp[q * d.mp + i]);
        const d2 ax = csub(csub(yo, cscale(mi, imu)), gv);
        d2 cc = cadd(ax, cscale(mi, imu));
        double dd = sqrt(cabs2(cc));
        if (dd == 0.0) {   // ArgMinY d2zero() guard (:516-520 / :524-528)
            cc = make_double2(1.0, 0.0);
            dd = 1.0;
        }
        const double f = (bi / dd + mu) / (1.0 + mu);
        y = cscale(cc, f);
        const d2 jv = csub(ax, y);
        reinterpret_cast<d2*>(a.AX)[om + i] = ax;
        reinterpret_cast<d2*>(a.M)[om + i] = cadd(mi, cscale(jv, mu));
        reinterpret_cast<d2*>(a.Yn)[om + i] = y;
        dy = csub(y, yo);
        const double aax = sqrt(cabs2(ax)) - bi;
        sv[0] = aax * aax;
        sv[1] = cabs2(ax);
        sv[2] = cabs2(y);
        sv[3] = cabs2(jv);
        sv[4] = cabs2(dy);
        sv[5] = fmax(fabs(gv.x), fabs(gv.y));
        sv[6] = fmax(fabs(y.x), fabs(y.y));
        sv[7] = fmax(fabs(dy.x), fabs(dy.y));
        sv[8] = 0.0 * (fabs(gv.x) + fabs(gv.y));
        sv[9] = 0.0 * (fabs(y.x) + fabs(y.y));
        sv[10] = 0.0 * (fabs(dy.x) + fabs(dy.y));
    }
    __syncthreads();   // every thread has read grow / cp
    if (iv) {
        Ts[i] = gv;
        grow[i] = y;
        cp[i] = dy;
    } else if (i < d.mp) {
        Ts[i] = d2zero();
        grow[i] = d2zero();
        cp[i] = d2zero();
    }
#pragma unroll
    for (int k = 0; k < 11; ++k) sv[k] = (k >= 5 && k < 8) ? wave_max(sv[k]) : wave_sum(sv[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 11; ++k) red[w][k] = sv[k];
    __syncthreads();
    double tot[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) {   // fixed order over the waves; every thread gets the same totals
        double v = red[0][k];
        for (int q = 1; q < 4; ++q) v = (k >= 5 && k < 8) ? fmax(v, red[q][k]) : v + red[q][k];
        tot[k] = v;
    }
    const bool imp = sqrt(tot[0]) < rs->opt_obj;   // iter_control makes the same decision (opt_Y here)
    if (iv && !a.yn_id && imp) reinterpret_cast<d2*>(a.optY)[om + i] = y;
    double p2v[3], scv[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) plane_scale(tot[5 + r] + tot[8 + r], c, p2v[r], scv[r]);
    __syncthreads();   // every thread has read red (reused below) and the opt_Y decision inputs
    if (t == 0) {
        rs->obj2 = tot[0];
        rs->nAX2 = tot[1];
        rs->nY2 = tot[2];
        rs->nJM2 = tot[3];
        rs->dY2 = tot[4];
        if (a.yn_id) rs->optysrc = imp ? a.yn_id : (oys == a.yn_id ? 0 : oys);
    }

    PSTAMP(3);
    // ---- digit planes of g, Y_new, dY (right-hand sides 0, 1, 2; slot 3 d2zero()) over the m inputs
    for (int e = t; e < 4 * 4 * d.nksH; e += PNT) {
        const int r = e / (4 * d.nksH), g4 = e - r * 4 * d.nksH;
        const d2* src = r == 0 ? Ts : (r == 1 ? grow : cp);
        d2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = (r < 3 && 4 * g4 + u < m) ? src[4 * g4 + u] : d2zero();
        const double p2r = r == 0 ? p2v[0] : (r == 1 ? p2v[1] : (r == 2 ? p2v[2] : 1.0));   // (no dynamic register index)
        put_digits4(Ad, [&](int tt) { return lds_row(r, tt) * L.rstH; }, 4 * g4, v, p2r);
    }
    __syncthreads();
    PSTAMP(4);

    // ---- W = c A^H g and the dual terms on the int8 matrix cores: rows = (right-hand side, digit),
    // codebook operand expanded from the A^H codes, one 32-column output tile per pass
    {
        i4v af[16];
        const int8_t* arow = Ad + (lane & 31) * L.rstH + 16 * (lane >> 5);
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) af[ks] = ks < d.nksH ? *reinterpret_cast<const i4v*>(arow + 32 * ks) : i4v{0, 0, 0, 0};
        const bool im = lane & 1;
        const uint32_t lutX = im ? LUT_NQ : LUT_P, lutY = im ? LUT_P : LUT_Q;   // conj(a) g: (p x + q y, p y - q x)
        double* Wb = a.W + (long long)b * 2 * n;
        double dacc = 0.0, nacc = 0.0;
        auto tile = [&](const uint4 (&cw)[2], int ct) {
            i16v acc = i16v{};
#pragma unroll
            for (int ks = 0; ks < 16; ++ks) {
                if (ks < d.nksH) {
                    const uint4 g = cw[ks >> 3];
                    const int j = (ks & 7) >> 1;
                    const uint32_t dw = j == 0 ? g.x : (j == 1 ? g.y : (j == 2 ? g.z : g.w));
                    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[ks], code_frag(dw, ks & 1, lutX, lutY), acc, 0, 0, 0);
                }
            }
            // lanes 0..31: slots 0 (g) and 2 (dY); lanes 32..63: slot 1 (Y_new).  Straight-line, so
            // that the compiler keeps both accumulators in registers (no lane-indexed selection)
            const int col = 32 * ct + (lane & 31);
            const bool lo = lane < 32, in = col < 2 * n;
            const double v0 = (lo ? scv[0] : scv[1]) * recombine(acc, 0), v1 = scv[2] * recombine(acc, 1);
            if (lo && in) Wb[col] = v0;
            dacc += (lo && in) ? v1 * v1 : 0.0;
            nacc += (!lo && in) ? v0 * v0 : 0.0;
        };
        for (int ct = w; ct < d.nctH; ct += 12) {   // codes three column tiles ahead
            cload(cq2, ct + 8);
            tile(cq0, ct);
            cload(cq0, ct + 12);
            if (ct + 4 < d.nctH) tile(cq1, ct + 4);
            cload(cq1, ct + 16);
            if (ct + 8 < d.nctH) tile(cq2, ct + 8);
        }
        dacc = wave_sum(dacc);
        nacc = wave_sum(nacc);
        if (lane == 0) {
            red[w][0] = dacc;
            red[w][1] = nacc;
        }
    }
    __syncthreads();
    if (t == 0) {
        double dv = red[0][0], nv = red[0][1];
        for (int q = 1; q < 4; ++q) {
            dv += red[q][0];
            nv += red[q][1];
        }
        rs->dAtY = dv;   // ||A^H (Y - Y0)||^2
        rs->nAtY = nv;   // ||A^H Y||^2
    }
    PSTAMP(5);
    PSTAMP_PRINT("pgk A|B|Ystep|digits|AH:", 6);
}

}  // namespace

// ---- host side -----------------------------------------------------------------------------
size_t pc_codes_bytes(int m, int n) {   // per realisation: A^H image, A image, row-major codes
    const PcDims d = pc_dims(m, n);
    return (size_t)d.nctH * d.nkgH * 512 + (size_t)d.nctA * d.nkgA * 512 + (size_t)m * d.nwR * 4;
}
// scratch (complex elements) of pc_inv_rec for an s x s block: F, F^H, T of this level + the deeper one
static long long pc_inv_scratch(int s) {
    if (s <= 32) return 0;
    const int h = 32 * ((s / 32) / 2), r = s - h;
    return 3LL * r * h + std::max(pc_inv_scratch(h), pc_inv_scratch(r));
}
// the matrix (mp32 x mp32) and the recursion's scratch
size_t pc_gw_bytes(int m) {
    const PcDims d = pc_dims(m, 16);
    return 16 * ((size_t)d.mp32 * d.mp32 + (size_t)pc_inv_scratch(d.mp32));
}
size_t pc_gt_bytes(int m) { const PcDims d = pc_dims(m, 16); return (size_t)d.ntile * 256 * 16; }
size_t pc_codesA_off(int batch, int m, int n) { const PcDims d = pc_dims(m, n); return (size_t)batch * d.nctH * d.nkgH * 128; }
bool pc_supported(int m, int n) { return m >= 1 && m <= PC_MAXM && n >= 1 && n <= PC_MAXN && pgk_lds(m, n).total <= 64 * 1024; }

void launch_pc_pack(int batch, int m, int n, const double* A, double* cb, uint32_t* codes, int* flag, hipStream_t st) {
    const PcDims d = pc_dims(m, n);
    uint32_t* cH = codes;
    uint32_t* cA = cH + (size_t)batch * d.nctH * d.nkgH * 128;
    uint32_t* cR = cA + (size_t)batch * d.nctA * d.nkgA * 128;
    if (!lds_fits(reinterpret_cast<const void*>(&pc_pack_kernel), "pc_pack_kernel", (size_t)32 * 16 * d.nksA)) return;
    hipLaunchKernelGGL(pc_pack_kernel, dim3(batch, d.nb32), dim3(PNT), (size_t)32 * 16 * d.nksA, st, m, n, A, cb, cH,
                       cA, cR, flag);
}

// H^{-1} in place for the s x s Hermitian block at H (leading dimension ld, realisation stride hs,
// complex elements) of nb realisations; scr: scratch with realisation stride ss (complex)
static void pc_inv_rec(int nb, int s, double* H, int ld, long long hs, double* scr, long long ss, hipStream_t st) {
    if (s <= 32) {
        hipLaunchKernelGGL(inv32_kernel, dim3(nb), dim3(PNT), 0, st, ld, hs, H);
        return;
    }
    const int h = 32 * ((s / 32) / 2), r = s - h;
    double* A = H;
    double* B = H + 2 * (size_t)h * ld;       // rows h.., columns 0..h
    double* D = B + 2 * (size_t)h;            // rows h.., columns h..
    double* Up = H + 2 * (size_t)h;           // rows 0..h, columns h..
    double* F = scr;                          // r x h
    double* Fh = F + 2 * (size_t)r * h;       // h x r
    double* T = Fh + 2 * (size_t)h * r;       // h x r
    double* next = T + 2 * (size_t)h * r;
    pc_inv_rec(nb, h, A, ld, hs, next, ss, st);
    // F = B A^{-1} = B (A^{-1})^H                                 (C = V L^H with V = B, L = A^{-1})
    launch_zgemm(0, true, h, h, r, A, ld, hs, B, ld, hs, F, nullptr, h, ss, nb, st);
    hipLaunchKernelGGL(ctrans_kernel<false>, dim3((h + 31) / 32, (r + 31) / 32, nb), dim3(PNT), 0, st, r, h, F, ss,
                       nullptr, 0, Fh, r, ss);
    // S = D - F B^H (in place)
    launch_zgemm(1, true, r, h, r, B, ld, hs, F, h, ss, D, D, ld, hs, nb, st);
    pc_inv_rec(nb, r, D, ld, hs, next, ss, st);
    // T = F^H S^{-1}; A^{-1} + T F = A^{-1} + T (F^H)^H; off-diagonal blocks -T, -T^H
    launch_zgemm(0, true, r, r, h, D, ld, hs, Fh, r, ss, T, nullptr, r, ss, nb, st);
    launch_zgemm(2, true, h, r, h, Fh, r, ss, T, r, ss, A, A, ld, hs, nb, st);
    hipLaunchKernelGGL(ctrans_kernel<true>, dim3((r + 31) / 32, (h + 31) / 32, nb), dim3(PNT), 0, st, h, r, T, ss,
                       Up, ld, B, ld, hs);
}

static bool pc_use_gj() {   // ACE_PC_GJ=1: the blocked Gauss-Jordan of r01 (A/B comparisons)
    static const bool v = [] {
        const char* e = exp_env("ACE_PC_GJ");
        return e && e[0] == '1';
    }();
    return v;
}

void launch_pc_ginv(int batch, int m, int n, const uint32_t* codes, const double* cb, double* Gw, double* Gt,
                    hipStream_t st) {
    if (!pc_use_gj()) {
        const PcDims d = pc_dims(m, n);
        const uint32_t* cR = codes + (size_t)batch * d.nctH * d.nkgH * 128 + (size_t)batch * d.nctA * d.nkgA * 128;
        const long long s2 = (long long)d.mp32 * d.mp32;   // complex elements per matrix
        // matrices [batch][mp32][mp32], then the scratch [batch][pc_inv_scratch]
        double* scr = Gw + 2 * s2 * batch;
        const long long ss = std::max(1LL, pc_inv_scratch(d.mp32));
        hipLaunchKernelGGL(pc_k_kernel, dim3(batch, d.nb32 * (d.nb32 + 1) / 2), dim3(PNT), (size_t)64 * (d.nwR + 1) * 4,
                           st, m, n, cR, cb, Gw);
        pc_inv_rec(batch, d.mp32, Gw, d.mp32, s2, scr, ss, st);
        hipLaunchKernelGGL(pc_tiles_kernel, dim3(batch, d.ntile), dim3(PNT), 0, st, m, Gw, Gt);
        return;
    }
    const PcDims d = pc_dims(m, n);
    const uint32_t* cR = codes + (size_t)batch * d.nctH * d.nkgH * 128 + (size_t)batch * d.nctA * d.nkgA * 128;
    static const int chunk_env = [] {
        const char* e = exp_env("ACE_PC_CHUNK");
        return e ? atoi(e) : 0;
    }();
    const int chunk = chunk_env > 0 ? chunk_env : batch;
    const size_t gws = (size_t)2 * d.mp32 * d.mp32, gts = (size_t)d.ntile * 512;
    for (int b0 = 0; b0 < batch; b0 += chunk) {
        const int nb = std::min(chunk, batch - b0);
        double* Gwc = Gw + gws * b0;
        hipLaunchKernelGGL(pc_k_kernel, dim3(nb, d.nb32 * (d.nb32 + 1) / 2), dim3(PNT), (size_t)64 * (d.nwR + 1) * 4,
                           st, m, n, cR + (size_t)b0 * m * d.nwR, cb + b0, Gwc);
        for (int k = 0; k < d.nb32; ++k) {
            hipLaunchKernelGGL(gj_panel_kernel, dim3(nb), dim3(PNT), 0, st, d.mp32, k, Gwc);
            if (d.nb32 > 1) hipLaunchKernelGGL(gj_update_kernel, dim3(nb, d.nb32 - 1), dim3(PNT), 0, st, d.mp32, k, Gwc);
        }
        hipLaunchKernelGGL(pc_tiles_kernel, dim3(nb, d.ntile), dim3(PNT), 0, st, m, Gwc, Gt + gts * b0);
    }
}

void launch_pc_apply_a(int batch, int m, int n, const uint32_t* codesA, const double* cb, const double* X0, double* P0,
                       hipStream_t st) {
    const PcDims d = pc_dims(m, n);
    const size_t lds = ((16 * (size_t)d.mp + 15) & ~(size_t)15) + 8 * (size_t)(32 * d.nksA + 16);
    if (!lds_fits(reinterpret_cast<const void*>(&pc_apply_a_kernel), "pc_apply_a_kernel", lds)) return;
    hipLaunchKernelGGL(pc_apply_a_kernel, dim3(batch), dim3(PNT), lds, st, m, n, codesA, cb, X0, P0);
}

void launch_pgk(int batch, const PgkArgs& a, hipStream_t st) {
    const size_t lds = (size_t)pgk_lds(a.m, a.n).total;
    if (!lds_fits(reinterpret_cast<const void*>(&pgk_kernel), "pgk_kernel", lds)) return;
    hipLaunchKernelGGL(pgk_kernel, dim3(batch), dim3(PNT), lds, st, a);
}

}  // namespace ace
