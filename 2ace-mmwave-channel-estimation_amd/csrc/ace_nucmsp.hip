// A2nuclear InferADMM at r = 1 on one shared sensing matrix, iterated in m-space
// (inferLowRank_Nuclear.m:269-383 with the Z-prox of :411-439).
//
// At r = 1 the nuclear Z-prox is a scaling, Z' = s E with s = max(0, ||E|| - 1/mu) / ||E||
// (Shrink of the one singular value of the n x 1 iterate), E = X + N/mu.  Then
//   N' = N + mu (X - Z') = mu (E - Z') = mu (1 - s) E,
// so after every iteration Z and N are both multiples of the same n-vector E, which stays in
// span{X_init} + range(A^H).  The state is E_prev = alpha X_init + A^H e (a real scalar and one
// m-vector e) with its image A E_prev, and the two multiples Z = a_z E_prev, N = a_n E_prev:
//   init (:309): E_prev = X_init (alpha = 1, e = 0), a_z = the prox scale at mu = 1, a_n = 0;
//   V = Z - N/mu = c_v E_prev (c_v = a_z - a_n/mu),  A V = c_v A E_prev   (A E_0 = P0 = A X_init)
//   T = (Y - M/mu) - A V,  g = G T (ArgMinX in Woodbury form),  K g = T - g    ((I + K) G = I)
//   X = c_v E_prev + A^H g,   E_new = X + N/mu = a_z E_prev + A^H g:
//       e_new = a_z e + g,  A E_new = a_z A E_prev + K g,  alpha_new = a_z alpha
//   s = Shrink(||E_new||),  a_z' = s,  a_n' = mu (1 - s).
// The norms of the convergence test (:364-370: ||X||, ||Z'||, ||X - Z'||, ||Z' - Z||) are
// quadratic forms in ||E_prev||^2 (carried), <E_prev, A^H g> = Re((A E_prev)^H g) and
// ||A^H g||^2 = Re(g^H K g), reduced per realisation in a fixed order.  The Y-step (:326-337) is
// the reference's, on AX = (Y - M/mu) - g.  The dual terms ||A^H (Y - Y0)||^2 and ||A^H Y||^2 are
// formed only when the test needs them (lazy dual residual), here on the f64
// matrix cores with K in fragment order.  The best iterate is kept as (opt_a, opt_w) with
// X = c_v alpha X_init + A^H (c_v e + g), materialised once after the loop.
//
// One launch per iteration and 16 realisations per 512-thread work-group, as gyk_kernel
// (ace_i8gemm.hip): T in LDS, g = G T on v_mfma_f64_16x16x4_f64 (3M form, G streamed from L2 in
// fragment order), then the Y-step and the E update on each lane's 2 x 4 outputs; a second pass
// only for realisations whose iterate is recorded.  Per realisation and iteration it moves Y, M,
// B, e, A E in and Y', M', e', A E' out (no n-vector at all) and runs 8 m^2 flops on the
// matrix cores.  In exact arithmetic this is the reference iteration; in floating point the
// products are formed in another order (the nuclear refinement is rounding-chaotic beyond ~60
// iterations: DESIGN §6).
#include "ace_common.hpp"
#include "ace_zcommon.hpp"

namespace ace {

namespace {
constexpr int NT = 512;    // threads per work-group (8 waves)
constexpr int GRB = 16;    // realisations per work-group (one f64 MFMA row tile)
constexpr int GSK = 4;     // f64 K-steps (4 complex each) per pipeline stage
__host__ __device__ __forceinline__ int nms_mp(int m) { return (m + 31) & ~31; }

struct GSet {
    d2 f[GSK][2];
};
struct TSet {
    d2 v[GSK];
};

// P[c][r] (3M accumulators) of the lane's 2 x 4 outputs of  out_i = sum_k L[i][k] v_k  for the
// 16 realisation rows held in LDS (Ts, row stride tst), L in fragment order (launch_gyk_gfrag).
__device__ __forceinline__ void frag_mv(const d2* __restrict__ Lf, const d2* Ts, int tst, int mp, int lane, int w,
                                        d4v (&p1)[2], d4v (&p2)[2], d4v (&p3)[2]) {
    const int nct = mp / 16, nks = mp / 4, nstage = nks / GSK;
    const int ct0 = min(2 * w, nct - 1), ct1 = min(2 * w + 1, nct - 1);
    const d2* gp0 = Lf + (long long)ct0 * 64 + lane;
    const d2* gp1 = Lf + (long long)ct1 * 64 + lane;
    auto gload = [&](GSet& gs, int s) {
#pragma unroll
        for (int kk = 0; kk < GSK; ++kk) {
            const long long ks = min(GSK * s + kk, nks - 1);
            gs.f[kk][0] = gp0[ks * nct * 64];
            gs.f[kk][1] = gp1[ks * nct * 64];
        }
    };
    const d2* trow = Ts + (lane & 15) * tst + (lane >> 4);
    auto tload = [&](TSet& ts, int s) {
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
#pragma unroll
    for (int c = 0; c < 2; ++c) p1[c] = p2[c] = p3[c] = d4v{0.0, 0.0, 0.0, 0.0};
    GSet gA, gB;
    TSet tA, tB;
    gload(gA, 0);
    tload(tA, 0);
    for (int s = 0; s < nstage; s += 2) {   // nstage is even (mp a multiple of 32)
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
__device__ __forceinline__ d2 frag_out(const d4v (&p1)[2], const d4v (&p2)[2], const d4v (&p3)[2], int c, int r) {
    const double e1 = p1[c][r], e2 = p2[c][r];
    return make_double2(e1 - e2, p3[c][r] - e1 - e2);
}
__device__ __forceinline__ double cdotr(d2 a, d2 b) { return a.x * b.x + a.y * b.y; }   // Re(conj(a) b)

constexpr int NSUM = 7;    // Y-step: obj2 nAX2 nY2 nJM2 dY2; m-space: <E_prev, A^H g>, ||A^H g||^2

// FIN: only finish the convergence tests the last iteration left pending (no iteration).
template <bool FIN>
__global__ __launch_bounds__(NT, 1) void nms_kernel(int nb, int m, NmsArgs a, ZArgs za) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ double red[8][GRB][NSUM];
    __shared__ int live_s[GRB], pend_s[GRB], imp_s[GRB], cur_s[GRB];
    __shared__ double mu_s[GRB], al_s[GRB], az_s[GRB], an_s[GRB], s_s[GRB];
    const int mp = nms_mp(m), tst = mp + 1, nct = mp / 16;
    d2* Ts = reinterpret_cast<d2*>(smem);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, j0 = blockIdx.x * GRB;
    if (t < GRB) {
        const int j = j0 + t;
        const bool lv = j < nb && !a.rs[j].done;
        live_s[t] = lv;
        pend_s[t] = lv && a.rs[j].dpend;
        mu_s[t] = lv ? a.rs[j].mu : 1.0;
        al_s[t] = lv ? a.rs[j].na : 0.0;
        az_s[t] = lv ? a.rs[j].naz : 0.0;
        an_s[t] = lv ? a.rs[j].nbeta : 0.0;
    }
    __syncthreads();
    // ---- pending convergence tests of the previous iteration: ||A^H Y_k||^2 = Y_k^H K Y_k and
    // ||A^H (Y_k - Y_{k-1})||^2 (Y_k in Yo, Y_{k-1} still in Yn), then the test and the mu update
    if (__syncthreads_or(t < GRB && pend_s[t])) {
        for (int pass = 0; pass < 2; ++pass) {
            for (int idx = t; idx < GRB * tst; idx += NT) {
                const int jl = idx / tst, k = idx - jl * tst;
                d2 v = make_double2(0.0, 0.0);
                if (k < m && pend_s[jl]) {
                    const long long o = (long long)(j0 + jl) * m + k;
                    const d2 yk = reinterpret_cast<const d2*>(a.Yo)[o];
                    v = pass ? csub(yk, reinterpret_cast<const d2*>(a.Yn)[o]) : yk;
                }
                Ts[idx] = v;
            }
            __syncthreads();
            d4v p1[2], p2[2], p3[2];
            frag_mv(reinterpret_cast<const d2*>(a.Kf), Ts, tst, mp, lane, w, p1, p2, p3);
            double q[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int jl = (lane >> 4) + 4 * r, i = 16 * (2 * w + c) + (lane & 15);
                    if (2 * w + c < nct && i < m) q[r] += cdotr(Ts[jl * tst + i], frag_out(p1, p2, p3, c, r));
                }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                q[r] = bsum16(q[r]);
                if ((lane & 15) == 0) red[w][(lane >> 4) + 4 * r][pass] = q[r];
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
            if (dual_finish(a.dc, rs, dv, nv)) live_s[t] = 0;
            mu_s[t] = rs->mu;
        }
        __syncthreads();
    }
    if constexpr (FIN) return;

    // ---- T = (Y - M/mu) - A V,  V = c_v E_prev, formed on this lane's pass-1 outputs (realisation
    // (lane >> 4) + 4 r, entry 16 (2 w + c) + (lane & 15)): Y and M stay in registers for the Y-step instead
    // of being read again after G T (by then other work-groups' streams have evicted them from the L2)
    d2 yh[2][4], mh[2][4];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int ct = 2 * w + c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int jl = (lane >> 4) + 4 * r, i = 16 * ct + (lane & 15);
            const bool in = ct < nct && i < m && live_s[jl];
            const long long o = (long long)(live_s[jl] ? j0 + jl : j0) * m + min(i, m - 1);   // (clamped: loads
            const d2 y = reinterpret_cast<const d2*>(a.Yo)[o], mm = reinterpret_cast<const d2*>(a.M)[o];   //  batched)
            const d2 aep = reinterpret_cast<const d2*>(a.AEo)[o];
            yh[c][r] = y;
            mh[c][r] = mm;
            d2 v = make_double2(0.0, 0.0);
            if (in) {
                const double imu = 1.0 / mu_s[jl], cv = az_s[jl] - an_s[jl] * imu;
                v = make_double2(fma(-mm.x, imu, y.x) - cv * aep.x, fma(-mm.y, imu, y.y) - cv * aep.y);
            }
            if (ct < nct) Ts[jl * tst + i] = v;
        }
    }
    if (t < GRB) Ts[t * tst + mp] = make_double2(0.0, 0.0);   // (the row stride's pad column)
    __syncthreads();
    // ---- g = G T
    d4v p1[2], p2[2], p3[2];
    frag_mv(reinterpret_cast<const d2*>(a.Gf), Ts, tst, mp, lane, w, p1, p2, p3);

    // ---- pass 1: the Y-step, E_new = a_z E_prev + A^H g as (e_new, K e_new), and the sums
    double v[4][NSUM];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < NSUM; ++k) v[r][k] = 0.0;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int ct = 2 * w + c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int jl = (lane >> 4) + 4 * r, i = 16 * ct + (lane & 15);
            if (ct >= nct || i >= m || !live_s[jl]) continue;
            const long long off = (long long)(j0 + jl) * m + i;
            const d2 gv = frag_out(p1, p2, p3, c, r), tv = Ts[jl * tst + i];
            const double mu = mu_s[jl], imu = 1.0 / mu, az = az_s[jl];
            const d2 mii = mh[c][r], yo = yh[c][r];   // (read with T's inputs)
            const double Bi = a.B[off];
            // Y-step (:326-337), the reference's expressions
            const d2 ax = csub(csub(yo, cscale(mii, imu)), gv);
            d2 cc = cadd(ax, cscale(mii, imu));
            double d = sqrt(cabs2(cc));
            if (d == 0.0) {   // ArgMinY zero guard (:516-520 / :524-528)
                cc = make_double2(1.0, 0.0);
                d = 1.0;
            }
            const double f = (Bi / d + mu) / (1.0 + mu);
            const d2 y = cscale(cc, f);
            const d2 jv = csub(ax, y);
            reinterpret_cast<d2*>(a.M)[off] = cadd(mii, cscale(jv, mu));
            reinterpret_cast<d2*>(a.Yn)[off] = y;
            const double aax = sqrt(cabs2(ax)) - Bi;
            v[r][0] += aax * aax;
            v[r][1] += cabs2(ax);
            v[r][2] += cabs2(y);
            v[r][3] += cabs2(jv);
            v[r][4] += cabs2(csub(y, yo));
            // E_new = a_z E_prev + A^H g:  e_new = a_z e + g,  A E_new = a_z A E_prev + K g,  K g = T - g
            const d2 e = reinterpret_cast<const d2*>(a.Eo)[off], aep = reinterpret_cast<const d2*>(a.AEo)[off];
            const d2 kg = csub(tv, gv);
            reinterpret_cast<d2*>(a.En)[off] = make_double2(fma(az, e.x, gv.x), fma(az, e.y, gv.y));
            reinterpret_cast<d2*>(a.AEn)[off] = make_double2(fma(az, aep.x, kg.x), fma(az, aep.y, kg.y));
            v[r][5] += cdotr(aep, gv);   // <E_prev, A^H g> = Re((A E_prev)^H g)
            v[r][6] += cdotr(gv, kg);    // ||A^H g||^2 = Re(g^H K g)
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int k = 0; k < NSUM; ++k) v[r][k] = bsum16(v[r][k]);
        if ((lane & 15) == 0)
#pragma unroll
            for (int k = 0; k < NSUM; ++k) red[w][(lane >> 4) + 4 * r][k] = v[r][k];
    }
    __syncthreads();
    // ---- the Z-step of each realisation on one thread: prox, residual norms, control
    if (t < GRB) {
        int imp = 0, cur = 0;
        double cvo = 0.0;
        if (live_s[t]) {
            double q[NSUM];
#pragma unroll
            for (int k = 0; k < NSUM; ++k) q[k] = 0.0;
            for (int ww = 0; ww < 8; ++ww)   // fixed order over the waves
#pragma unroll
                for (int k = 0; k < NSUM; ++k) q[k] += red[ww][t][k];
            RealState& rs = a.rs[j0 + t];
            rs.obj2 = q[0];
            rs.nAX2 = q[1];
            rs.nY2 = q[2];
            rs.nJM2 = q[3];
            rs.dY2 = q[4];
            const double mu = mu_s[t], imu = 1.0 / mu, az = az_s[t], al = al_s[t];
            const double cv = az - an_s[t] * imu;        // V = Z - N/mu = c_v E_prev
            const double ne = rs.nep2, hp = q[5], hh = fmax(0.0, q[6]);
            // X = c_v E_prev + A^H g,  E = X + N/mu = a_z E_prev + A^H g,  Z' = s E (Shrink, :421-439)
            const double nE2 = fmax(0.0, az * az * ne + 2.0 * az * hp + hh);
            const double nE = sqrt(nE2);
            const double s = nE > 0.0 ? fmax(0.0, nE - imu) / nE : 0.0;
            const double nX2 = fmax(0.0, cv * cv * ne + 2.0 * cv * hp + hh);
            const double nZ2 = s * s * nE2;
            const double u = cv - s * az, u1 = 1.0 - s;   // X - Z' = u E_prev + (1 - s) A^H g
            const double jn2 = fmax(0.0, u * u * ne + 2.0 * u * u1 * hp + u1 * u1 * hh);
            const double wz = az * (s - 1.0);              // Z' - Z = wz E_prev + s A^H g
            const double dZ2 = fmax(0.0, wz * wz * ne + 2.0 * wz * s * hp + s * s * hh);
            const int ctl = iter_control_in(za, &rs, iter_in(&rs), mu, nX2, nZ2, jn2, dZ2, 0.0, 0.0);
            imp = ctl & 1;
            // Z' = s E_new, N' = N + mu (X - Z') = mu (1 - s) E_new  (E_new's X_init coefficient a_z alpha)
            rs.na = az * al;
            rs.naz = s;
            rs.nbeta = mu * (1.0 - s);
            rs.nep2 = nE2;
            if (imp) rs.nopt_a = cv * al;
            // the last iterate stands in for opt_X while no objective was finite (finalize's fallback)
            cur = !(rs.opt_obj < INFINITY);
            if (cur) rs.ncur_a = cv * al;
            cvo = cv;
        }
        imp_s[t] = imp;
        cur_s[t] = cur;
        s_s[t] = cvo;
    }
    __syncthreads();
    // ---- pass 2 (realisations whose iterate is recorded): X's m-part c_v e + g, opt_Y
    if (!__syncthreads_or(t < GRB && (imp_s[t] || cur_s[t]))) return;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int ct = 2 * w + c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int jl = (lane >> 4) + 4 * r, i = 16 * ct + (lane & 15);
            if (ct >= nct || i >= m || !live_s[jl] || !(imp_s[jl] || cur_s[jl])) continue;
            const long long off = (long long)(j0 + jl) * m + i;
            const d2 gv = frag_out(p1, p2, p3, c, r), e = reinterpret_cast<const d2*>(a.Eo)[off];
            const double cv = s_s[jl];
            const d2 x = make_double2(fma(cv, e.x, gv.x), fma(cv, e.y, gv.y));
            if (imp_s[jl]) {
                reinterpret_cast<d2*>(a.optW)[off] = x;
                reinterpret_cast<d2*>(a.optY)[off] = reinterpret_cast<const d2*>(a.Yn)[off];
            }
            if (cur_s[jl]) reinterpret_cast<d2*>(a.curW)[off] = x;
        }
    }
}

// P0 = A X_init is formed by the caller; here E_prev = X_init (alpha = 1, e = 0, A E_prev = P0), Z = a_z E_prev
// with a_z the prox scale at mu = 1 (:309, Z = ArgMinZ(X, 0, 1)), N = 0 (a_n = 0), ||E_prev||^2.
__global__ __launch_bounds__(256) void nms_init_kernel(int n, int m, const double* __restrict__ Xi, NmsArgs a) {
    __shared__ double red[16];
    const int b = blockIdx.x;
    const d2* x = reinterpret_cast<const d2*>(Xi) + (long long)b * n;
    double s[1] = {0.0};
    for (int k = threadIdx.x; k < n; k += blockDim.x) s[0] += cabs2(x[k]);
    block_sum<1>(s, red);
    const long long o = (long long)b * m;
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        reinterpret_cast<d2*>(a.Eo)[o + i] = make_double2(0.0, 0.0);
        reinterpret_cast<d2*>(a.AEo)[o + i] = reinterpret_cast<const d2*>(a.P0)[o + i];   // A E_prev = A X_init
    }
    if (threadIdx.x == 0) {
        RealState& rs = a.rs[b];
        const double nz = sqrt(s[0]);
        rs.nx0 = s[0];
        rs.nep2 = s[0];
        rs.na = 1.0;
        rs.naz = nz > 0.0 ? fmax(0.0, nz - 1.0) / nz : 0.0;
        rs.nbeta = 0.0;
        rs.nopt_a = 0.0;
        rs.ncur_a = 0.0;
        rs.dpend = 0;
    }
}

// The output iterate's parts: V[b] = a X_init (a = opt_a, or the last iterate's while no objective
// was finite) and Wsel[b] = opt_w / cur_w; the caller adds A^H Wsel.
__global__ __launch_bounds__(256) void nms_out_kernel(int n, int m, const double* __restrict__ Xi, NmsArgs a,
                                                      double* __restrict__ V, double* __restrict__ Wsel) {
    const int b = blockIdx.x;
    const RealState& rs = a.rs[b];
    const bool have = rs.opt_obj < INFINITY;
    const double co = have ? rs.nopt_a : rs.ncur_a;
    const d2* x = reinterpret_cast<const d2*>(Xi) + (long long)b * n;
    d2* v = reinterpret_cast<d2*>(V) + (long long)b * n;
    for (int k = threadIdx.x; k < n; k += blockDim.x) v[k] = cscale(x[k], co);
    const d2* src = reinterpret_cast<const d2*>(have ? a.optW : a.curW) + (long long)b * m;
    d2* dst = reinterpret_cast<d2*>(Wsel) + (long long)b * m;
    for (int i = threadIdx.x; i < m; i += blockDim.x) dst[i] = src[i];
}
}  // namespace

size_t nms_lds_bytes(int m) { return (size_t)GRB * (nms_mp(m) + 1) * sizeof(d2); }

void launch_nms(int nb, int m, const NmsArgs& a, const ZArgs& za, bool fin, hipStream_t st) {
    const size_t lds = nms_lds_bytes(m);
    const dim3 grid((nb + GRB - 1) / GRB);
    if (fin) {
        if (lds_fits(reinterpret_cast<const void*>(&nms_kernel<true>), "nms_kernel<fin>", lds))
            hipLaunchKernelGGL(nms_kernel<true>, grid, dim3(NT), lds, st, nb, m, a, za);
    } else if (lds_fits(reinterpret_cast<const void*>(&nms_kernel<false>), "nms_kernel", lds)) {
        hipLaunchKernelGGL(nms_kernel<false>, grid, dim3(NT), lds, st, nb, m, a, za);
    }
}
bool nms_supported(int m) {
    const size_t lds = nms_lds_bytes(m);
    return lds <= 64 * 1024 || (lds <= lds_dyn_budget(reinterpret_cast<const void*>(&nms_kernel<true>)) &&
                                lds <= lds_dyn_budget(reinterpret_cast<const void*>(&nms_kernel<false>)));
}
void launch_nms_init(int nb, int n, int m, const double* Xi, const NmsArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(nms_init_kernel, dim3(nb), dim3(256), 0, st, n, m, Xi, a);
}
void launch_nms_out(int nb, int n, int m, const double* Xi, const NmsArgs& a, double* V, double* Wsel, hipStream_t st) {
    hipLaunchKernelGGL(nms_out_kernel, dim3(nb), dim3(256), 0, st, n, m, Xi, a, V, Wsel);
}

}  // namespace ace
