// Work-group Hermitian eigensolver for matrices of order <= 32 held in LDS, shared by
// the four-wave Z-prox kernels (ace_zprox.hip: E E^H of the A2only ArgMinZ,
// inferLowRankV4_multi.m:428) and the r-column stage kernels (ace_stage.hip: the
// 32x32 E E^H at r > 1, the r x r Gram X^H X of the rotation at :263-264 and of the
// nuclear-norm prox, inferLowRank_Nuclear.m:415).
//
// Parallel cyclic Jacobi in the position frame: pair k always sits at positions
// (2k, 2k+1); after every step the positions are permuted by the circle-method map
// (circ_next), so each sweep of sz-1 steps meets every index pair once.  H lives in
// packed upper-triangular form, double buffered (read cur, write the permuted result
// to nxt) in the space of one 32x33 tile.  Q stays in label (original) order; Lab[.][p]
// is the label at position p.  All addressing is static per thread, so a step is
// branch-free with one barrier.  Stop: a pre-sweep test over all off-diagonals
// (|h_pq| <= 1e-18 tr H or |h_pq|^2 <= 1e-32 |h_pp h_qq|), so no confirming sweep runs.
#pragma once
#include "ace_zcommon.hpp"

namespace ace {
namespace {

constexpr int JAC_MAX_SWEEPS = 40;

struct JacobiShared {
    int flags[JAC_MAX_SWEEPS + 1];
    int Lab[2][ZT];
    double4 RotS[ZT / 2];
};

// Eigendecomposition of the Hermitian sz x sz matrix in H (full 32 x ZHS tile, sz even,
// 2 <= sz <= 32).  Q (32 x ZHS tile) holds the starting basis (identity, or a warm start
// whose columns are orthonormal) and on return its first sz columns are eigenvectors;
// wv[c] receives the eigenvalue of column c.  H is destroyed.  Must be called by all
// threads of a 256-thread block.  Returns the number of sweeps run (JAC_MAX_SWEEPS =
// not converged).
__device__ int jacobi_eig32(d2* H, d2* Q, int sz, double* wv, JacobiShared& sh) {
    const int t = threadIdx.x, lane = t & 63;
    if (t <= JAC_MAX_SWEEPS) sh.flags[t] = 0;
    __syncthreads();
    double tr = 0.0;
    for (int k = 0; k < sz; ++k) tr += fabs(H[k * ZHS + k].x);
    const double abs_tol = 1e-18 * tr;
    const int P = sz >> 1;
    {  // full tile -> packed upper triangle (buffer 0)
        const int j = t & 31, i0 = t >> 5;  // rows i0, i0+8, i0+16, i0+24 of column j
        const d2 h0 = H[i0 * ZHS + j], h1 = H[(i0 + 8) * ZHS + j];
        const d2 h2 = H[(i0 + 16) * ZHS + j], h3 = H[(i0 + 24) * ZHS + j];
        __syncthreads();
        if (i0 <= j) H[up_idx(i0, j)] = h0;
        if (i0 + 8 <= j) H[up_idx(i0 + 8, j)] = h1;
        if (i0 + 16 <= j) H[up_idx(i0 + 16, j)] = h2;
        if (i0 + 24 <= j) H[up_idx(i0 + 24, j)] = h3;
        if (t < ZT) sh.Lab[0][t] = t;
        __syncthreads();
    }
    // static per-thread 2x2 block (ta <= tb) of slot pairs: read / write slots, conj flags
    int ta = -1, tb = -1;
    if (t < 136) {
        ta = c_tri_a[t];
        tb = c_tri_b[t];
        if (tb >= P) ta = -1;
    }
    const int sa = ta < 0 ? 0 : ta, sb = tb < 0 ? 0 : tb;
    int rd[4], wr[4], dg[4], dgj[4];
    double wsg[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 2 * sa + (r >> 1), j = 2 * sb + (r & 1);
        rd[r] = i <= j ? up_idx(i, j) : up_idx(j, i);
        dg[r] = up_idx(i, i);   // diagonals of row i and column j (convergence test)
        dgj[r] = up_idx(j, j);
        const int ii = circ_next(sz, i), jj = circ_next(sz, j);
        wr[r] = ii <= jj ? up_idx(ii, jj) : up_idx(jj, ii);
        wsg[r] = ii <= jj ? 1.0 : -1.0;
    }
    const bool diagblk = (ta == tb);                // (2k+1, 2k) mirrors (2k, 2k+1): not stored
    const double rsg10 = diagblk ? -1.0 : 1.0;      // diagonal block reads (2k+1,2k) as conj
    const int kl = lane & 15;                       // rotation applied to Q by this lane
    const int rp = up_idx(2 * kl, 2 * kl), rq = up_idx(2 * kl + 1, 2 * kl + 1), rc = up_idx(2 * kl, 2 * kl + 1);
    const int pn = t < sz ? circ_next(sz, t) : 0;
    int cur = 0, sweeps = 0;
    for (; sweeps < JAC_MAX_SWEEPS; ++sweeps) {
        if (ta >= 0) {  // convergence pre-check over this thread's off-diagonal entries
            const d2* Hc = H + cur * ZPACK;
            bool need = false;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool offd = !diagblk || r == 1;
                if (offd) need |= needs_rot(Hc[dg[r]].x, Hc[dgj[r]].x, Hc[rd[r]], abs_tol);
            }
            if (need) sh.flags[sweeps] = 1;
        }
        __syncthreads();
        if (!sh.flags[sweeps]) break;
        for (int s = 0; s < sz - 1; ++s) {
            const int nx = cur ^ 1;
            const d2* Hc = H + cur * ZPACK;
            d2* Hn = H + nx * ZPACK;
            if (t < P) {  // the step's rotations, once per work-group
                const Rot J = make_rot(Hc[rp].x, Hc[rq].x, Hc[rc], abs_tol);
                sh.RotS[t] = make_double4(J.cs, J.sn, J.e.x, J.e.y);
            }
            __syncthreads();
            const double4 ra = sh.RotS[sa], rb = sh.RotS[sb], rl = sh.RotS[kl];
            if (ta >= 0) {
                // H'[a,b] = Ja^H H[a,b] Jb,  J = [[cs, sn], [-sn e*, cs e*]]
                const d2 h00 = Hc[rd[0]], h01 = Hc[rd[1]], h11 = Hc[rd[3]];
                d2 h10 = Hc[rd[2]];
                h10.y *= rsg10;
                const d2 ebc = make_double2(rb.z, -rb.w);
                const d2 t01 = cmul(h01, ebc), t11 = cmul(h11, ebc);
                const d2 T00 = csub(cscale(h00, rb.x), cscale(t01, rb.y));
                const d2 T01 = cadd(cscale(h00, rb.y), cscale(t01, rb.x));
                const d2 T10 = csub(cscale(h10, rb.x), cscale(t11, rb.y));
                const d2 T11 = cadd(cscale(h10, rb.y), cscale(t11, rb.x));
                const d2 ea = make_double2(ra.z, ra.w);
                const d2 u10 = cmul(ea, T10), u11 = cmul(ea, T11);
                const d2 nv[4] = {csub(cscale(T00, ra.x), cscale(u10, ra.y)),
                                  csub(cscale(T01, ra.x), cscale(u11, ra.y)),
                                  cadd(cscale(T00, ra.y), cscale(u10, ra.x)),
                                  cadd(cscale(T01, ra.y), cscale(u11, ra.x))};
                Hn[wr[0]] = make_double2(nv[0].x, nv[0].y * wsg[0]);
                Hn[wr[1]] = make_double2(nv[1].x, nv[1].y * wsg[1]);
                Hn[wr[3]] = make_double2(nv[3].x, nv[3].y * wsg[3]);
                if (!diagblk) Hn[wr[2]] = make_double2(nv[2].x, nv[2].y * wsg[2]);
            }
            // Q <- Q J on label columns (Lab[2k], Lab[2k+1]) for (row i, pair k = lane & 15)
            if (kl < P) {
                const int lp = sh.Lab[cur][2 * kl], lq = sh.Lab[cur][2 * kl + 1];
                const d2 ebc = make_double2(rl.z, -rl.w);
                for (int e = t; e < ZT * 16; e += 256) {
                    const int i = e >> 4;
                    if (i < sz) {
                        const d2 qp = Q[i * ZHS + lp];
                        const d2 qq = cmul(Q[i * ZHS + lq], ebc);
                        Q[i * ZHS + lp] = csub(cscale(qp, rl.x), cscale(qq, rl.y));
                        Q[i * ZHS + lq] = cadd(cscale(qp, rl.y), cscale(qq, rl.x));
                    }
                }
            }
            if (t < sz) sh.Lab[nx][pn] = sh.Lab[cur][t];
            cur = nx;
            __syncthreads();
        }
    }
    // eigenvalue at position p belongs to eigenvector (Q column) Lab[p]
    if (t < sz) wv[sh.Lab[cur][t]] = H[cur * ZPACK + up_idx(t, t)].x;
    __syncthreads();
    return sweeps;
}

// 32x32 complex product from LDS tiles (row stride ZHS) on the f64 matrix cores:
// C (+)= opA(A) * opB(B), op = identity or conjugate transpose.  Wave w computes the
// 16x16 block rows [16*(w>>1), +16) x cols [16*(w&1), +16); real and imaginary
// parts accumulate in separate 16x16 f64 tiles (4 real MFMAs per complex k-step).
template <bool CTA, bool CTB>
__device__ __forceinline__ void mm32_acc(const d2* A, const d2* B, d4v& cr, d4v& ci, int lane, int w) {
    const int i0 = 16 * (w >> 1), j0 = 16 * (w & 1);
#pragma unroll
    for (int k0 = 0; k0 < 32; k0 += 4) {
        const int kk = k0 + (lane >> 4);
        d2 av = CTA ? A[kk * ZHS + i0 + (lane & 15)] : A[(i0 + (lane & 15)) * ZHS + kk];
        d2 bv = CTB ? B[(j0 + (lane & 15)) * ZHS + kk] : B[kk * ZHS + j0 + (lane & 15)];
        if (CTA) av.y = -av.y;
        if (CTB) bv.y = -bv.y;
        cr = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.x, cr, 0, 0, 0);
        cr = __builtin_amdgcn_mfma_f64_16x16x4f64(-av.y, bv.y, cr, 0, 0, 0);
        ci = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.y, ci, 0, 0, 0);
        ci = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bv.x, ci, 0, 0, 0);
    }
}
template <bool CTA, bool CTB>
__device__ __forceinline__ void mm32(const d2* A, const d2* B, d4v& cr, d4v& ci, int lane, int w) {
    cr = d4v{0.0, 0.0, 0.0, 0.0};
    ci = d4v{0.0, 0.0, 0.0, 0.0};
    mm32_acc<CTA, CTB>(A, B, cr, ci, lane, w);
}
// store an mm32 result: lane l, reg r -> row i0 + (l>>4) + 4r, col j0 + (l&15)
__device__ __forceinline__ void store32(d2* C, const d4v& cr, const d4v& ci, int lane, int w) {
    const int i0 = 16 * (w >> 1), j0 = 16 * (w & 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) C[(i0 + (lane >> 4) + 4 * r) * ZHS + j0 + (lane & 15)] = make_double2(cr[r], ci[r]);
}

// LAPACK's ascending eigenvalue order (ties by column index): asc[c] = position of column c.
__device__ __forceinline__ void ascending_positions(const double* wv, int sz, int* asc) {
    const int t = threadIdx.x;
    if (t < sz) {
        const double wk = wv[t];
        int p = 0;
        for (int j = 0; j < sz; ++j) p += (wv[j] < wk) || (wv[j] == wk && j < t);
        asc[t] = p;
    }
    __syncthreads();
}

}  // namespace
}  // namespace ace
