// PhaseLift (main/src/my_recovery_algorithms/MyPhaseLift.m:69-107): TFOCS's Auslender-
// Teboulle method on  min 0.5||diag(Phi X Phi^H) - b||^2 + lambda tr X,  X >= 0
// (solver_TraceLS.m, tfocs_AT.m:20-88, tfocs_backtrack.m, tfocs_iterate.m, prox_trace.m),
// batched over realisations that share one measurement matrix Phi (m x n).
//
// Reduced coordinates.  MyPhaseLift starts from X0 = 0 and every TFOCS iterate is built from
// prox outputs of  z_old - step * Phi^H diag(g) Phi, so by induction every x, y, z lies in
// { Q Xd Q^H } with Q an orthonormal basis of range(Phi^H) (d = rank Phi = m <= n).  With
// Phi^H = Q R (R = chol(Phi Phi^H), d x m):
//     A(X)  = diag(Phi X Phi^H) = diag(R^H Xd R),      A*(g) = Q (R diag(g) R^H) Q^H,
//     ||X||_F = ||Xd||_F,  <X, Y> = <Xd, Yd>,  eig(X) = eig(Xd) plus n - d zeros
// (the zeros fall below prox_trace's threshold and are dropped), so the whole iteration runs
// on d x d matrices exactly (in exact arithmetic; rounding differs from the dense n x n
// iteration at the 1e-15 level).  m > n (or a rank-deficient Phi) runs with Q = I, R = Phi^H.
//
// Per realisation the TFOCS scalars (L, theta, counters, backtracking switches) live in a
// PlState; each kernel below is one step of tfocs_AT.m's inner loop for the realisations
// still in it (act[b]), so realisations backtrack independently while the batched GEMMs
// (A, A*, prox assembly) run once for the whole batch.
#include "ace_common.hpp"
#include "ace_pipe.hpp"
#include "ace_phaselift.hpp"

namespace ace {

namespace {

__device__ __forceinline__ double block_sum1(double v, double* sh) {
    double a[1] = {v};
    block_sum<1>(a, sh);
    return a[0];
}

// TFOCS initialisation (tfocs_initialize.m): x0 = 0 -> A_x = 0, f_x = 0.5||b||^2, g_Ax = -b,
// y = z = x, theta = Inf, L = L0.  (The matrices and A vectors are zeroed by the host.)
__global__ __launch_bounds__(256) void pl_init_kernel(PlArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    __shared__ double red[16];
    const double* bv = a.bvec + (long long)b * a.m;
    double s = 0.0;
    for (int i = t; i < a.m; i += 256) {
        s += bv[i] * bv[i];
        a.gAy[(long long)b * a.m + i] = -bv[i];
        a.gAx[(long long)b * a.m + i] = -bv[i];
    }
    s = block_sum1(s, red);
    if (t == 0) {
        PlState p = {};
        p.L = a.L0;
        p.theta = INFINITY;
        p.f_x = 0.5 * s;
        p.f_y = p.f_x;
        p.C_x = 0.0;
        p.backtrack_simple = 1;
        p.have_gAy = 1;
        p.have_gAx = 1;
        p.have_gy = 0;
        a.st[b] = p;
    }
}

// tfocs_AT.m:22-31: x_old = x, A_x_old = A_x, z_old = z, A_z_old = A_z, L_old = L,
// L = L*alpha, theta_old = theta.
__global__ __launch_bounds__(256) void pl_outer_begin_kernel(PlArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    PlState& p = a.st[b];
    if (p.done) return;
    // x_old = x, z_old = z: 16-B accesses, four in flight per thread
    const long long n2 = (long long)a.d * a.d, o = b * n2;
    const d2* xs = reinterpret_cast<const d2*>(a.x) + o;
    const d2* zs = reinterpret_cast<const d2*>(a.z) + o;
    d2* xd = reinterpret_cast<d2*>(a.xo) + o;
    d2* zd = reinterpret_cast<d2*>(a.zo) + o;
    long long e = t;
    for (; e + 256 < n2; e += 512) {
        const d2 x0 = xs[e], x1 = xs[e + 256], z0 = zs[e], z1 = zs[e + 256];
        xd[e] = x0;
        xd[e + 256] = x1;
        zd[e] = z0;
        zd[e + 256] = z1;
    }
    for (; e < n2; e += 256) {
        xd[e] = xs[e];
        zd[e] = zs[e];
    }
    for (int i = t; i < a.m; i += 256) {
        a.Axo[(long long)b * a.m + i] = a.Ax[(long long)b * a.m + i];
        a.Azo[(long long)b * a.m + i] = a.Az[(long long)b * a.m + i];
    }
    __syncthreads();
    if (t == 0) {
        p.L_old = p.L;
        p.L = p.L * a.alpha;
        p.theta_old = p.theta;
        p.inner = 1;
    }
}

// tfocs_AT.m:33-45 (theta, the A_y counter) for every realisation still in its inner loop.
__global__ __launch_bounds__(256) void pl_theta_kernel(PlArgs a) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.batch) return;
    PlState& p = a.st[b];
    if (!p.inner || p.done) {
        a.act[b] = 0;
        return;
    }
    a.act[b] = 1;
    p.theta = 2.0 / (1.0 + sqrt(1.0 + 4.0 * (p.L / p.L_old) / (p.theta_old * p.theta_old)));
    p.ycomp = p.theta < 1.0;
    p.need_Ay = 0;
    if (p.ycomp) {
        if (p.cntr_Ay >= a.cntr_reset) {
            p.need_Ay = 1;
            p.cntr_Ay = 0.0;
        } else {
            p.cntr_Ay += 1.0;
        }
        p.f_y = INFINITY;
        p.have_gAy = 0;
        p.have_gy = 0;
    }
    atomicAdd(&a.cnt[0], 1);
    if (p.need_Ay) atomicAdd(&a.cnt[1], 1);
    if (!p.have_gy) atomicAdd(&a.cnt[4], 1);
}

// y = (1 - theta) x_old + theta z_old  (tfocs_AT.m:38)
__global__ __launch_bounds__(256) void pl_make_y_kernel(PlArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    const PlState& p = a.st[b];
    if (!a.act[b] || !p.ycomp) return;
    const double th = p.theta, om = 1.0 - th;
    const long long n2 = (long long)a.d * a.d, o = b * n2;   // (16-B accesses, the same expression per double)
    const d2* xo = reinterpret_cast<const d2*>(a.xo) + o;
    const d2* zo = reinterpret_cast<const d2*>(a.zo) + o;
    d2* y = reinterpret_cast<d2*>(a.y) + o;
    for (long long e = t; e < n2; e += 256) {
        const d2 u = xo[e], w = zo[e];
        y[e] = make_double2(om * u.x + th * w.x, om * u.y + th * w.y);
    }
}

// A_y = A(y) when the counter fired, else (1 - theta) A_x_old + theta A_z_old (tfocs_AT.m:39-44)
__global__ __launch_bounds__(256) void pl_set_Ay_kernel(PlArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    const PlState& p = a.st[b];
    if (!a.act[b] || !p.ycomp) return;
    const double th = p.theta, om = 1.0 - th;
    const long long o = (long long)b * a.m;
    for (int i = t; i < a.m; i += 256)
        a.Ay[o + i] = p.need_Ay ? a.Aex[o + i] : om * a.Axo[o + i] + th * a.Azo[o + i];
}

// smooth_quad at A_y - b (tfocs_AT.m:48-49); step = 1/(theta L), tau = lambda * step; and the
// gradient operand R o g_Ay for A*(g_Ay) = R diag(g) R^H (only where g_y is stale).
__global__ __launch_bounds__(256) void pl_grad_kernel(PlArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    __shared__ double red[16];
    PlState& p = a.st[b];
    if (!a.act[b]) return;
    const long long o = (long long)b * a.m;
    if (!p.have_gAy) {
        double s = 0.0;
        for (int i = t; i < a.m; i += 256) {
            const double g = a.Ay[o + i] - a.bvec[o + i];
            a.gAy[o + i] = g;
            s += g * g;
        }
        s = block_sum1(s, red);
        if (t == 0) {
            p.f_y = 0.5 * s;
            p.have_gAy = 1;
        }
    }
    if (!p.have_gy) {
        const d2* R = reinterpret_cast<const d2*>(a.R);
        d2* Pg = reinterpret_cast<d2*>(a.Pg) + (long long)b * a.d * a.m;
        for (long long e = t; e < (long long)a.d * a.m; e += 256) Pg[e] = cscale(R[e], a.gAy[o + e % a.m]);
    }
    __syncthreads();
    if (t == 0) {
        p.have_gy = 1;
        p.step = 1.0 / (p.theta * p.L);
        a.tau[b] = a.lambda * p.step;
    }
}

// prox_trace input (tfocs_AT.m:52-53, prox_trace.m:88-92): (W + W^H)/2, W = z_old - step g_y,
// written where the eigensolver reads its matrix.
__global__ __launch_bounds__(256) void pl_prox_in_kernel(PlArgs a) {
    // C = (W + W^H) / 2 with W = z_old - step G, by 32 x 32 tile pairs (I, J), (J, I) staged in LDS, so
    // every entry is read once and both tiles' reads and writes are row-coalesced (the element-wise form
    // read W[j][i] down a column: 7x the matrix bytes fetched).  Same expressions per entry.
    const int b = blockIdx.x, t = threadIdx.x;
    if (!a.act[b]) return;
    const double st = a.st[b].step;
    const int d = a.d, nt = (d + 31) / 32;
    const long long o = (long long)b * d * d;
    const d2* zo = reinterpret_cast<const d2*>(a.zo) + o;
    const d2* G = reinterpret_cast<const d2*>(a.G) + o;
    d2* C = reinterpret_cast<d2*>(a.scratch + (long long)b * a.hl.stride + a.hl.C);
    __shared__ d2 tu[32][33], tl[32][33];   // W(I, J) and W(J, I)
    const int cc = t & 31, r0 = t >> 5;      // column within the tile, first row (8 rows per pass)
    for (int I = 0; I < nt; ++I)
        for (int J = I; J < nt; ++J) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rr = r0 + 8 * q;
                const int i1 = 32 * I + rr, j1 = 32 * J + cc;   // W(I, J) entry (i1, j1)
                const int i2 = 32 * J + rr, j2 = 32 * I + cc;   // W(J, I) entry (i2, j2)
                if (i1 < d && j1 < d) {
                    const long long e = (long long)i1 * d + j1;
                    tu[rr][cc] = csub(zo[e], cscale(G[e], st));
                }
                if (i2 < d && j2 < d) {
                    const long long e = (long long)i2 * d + j2;
                    tl[rr][cc] = csub(zo[e], cscale(G[e], st));
                }
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rr = r0 + 8 * q;
                const int i1 = 32 * I + rr, j1 = 32 * J + cc;
                if (i1 < d && j1 < d) {   // C[i1][j1] from w1 = W[i1][j1], w2 = W[j1][i1]
                    const d2 w1 = tu[rr][cc], w2 = tl[cc][rr];
                    C[(long long)i1 * d + j1] = make_double2(0.5 * (w1.x + w2.x), 0.5 * (w1.y - w2.y));
                }
                const int i2 = 32 * J + rr, j2 = 32 * I + cc;
                if (I != J && i2 < d && j2 < d) {   // C[i2][j2] from W[i2][j2], W[j2][i2]
                    const d2 w1 = tl[rr][cc], w2 = tu[cc][rr];
                    C[(long long)i2 * d + j2] = make_double2(0.5 * (w1.x + w2.x), 0.5 * (w1.y - w2.y));
                }
            }
            __syncthreads();
        }
}

// prox_trace.m:140-147: keep s = lam - tau > 0; P = V^T diag(s), VT = V^T (zero beyond k), so
// z = P VT^H = V(:,tt) diag(s) V(:,tt)^H is one batched GEMM; C_z = lambda * sum(s).
__global__ __launch_bounds__(256) void pl_assemble_kernel(PlArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    if (!a.act[b]) return;
    const int d = a.d;
    const double* base = a.scratch + (long long)b * a.hl.stride;
    const int k = (int)base[a.hl.misc];
    const double tau = a.tau[b];
    const double sgn = base[a.hl.misc + 2] != 0.0 ? -1.0 : 1.0;   // (the complement side: s = tau - lam)
    const double* lam = base + a.hl.lam;
    const long long o = (long long)b * d * d;
    const d2* V = reinterpret_cast<const d2*>(a.V) + o;
    d2* P = reinterpret_cast<d2*>(a.P) + o;
    d2* VT = reinterpret_cast<d2*>(a.VT) + o;
    // VT[i][q] = V[q][i] (q < k, else 0) and P[i][q] = VT[i][q] (lam_q - tau), by 32 x 32 tiles through LDS: V read
    // along its rows (the element-wise form read V[q][i] down a column), the same values
    __shared__ d2 tv[32][33];
    // (column tiles past the kept count are all zero and not written: the assembly GEMM sums over q < k only)
    const int nt = (d + 31) / 32, ntq = (k + 31) / 32, cc = t & 31, r0 = t >> 5;
    for (int I = 0; I < nt; ++I)
        for (int Q = 0; Q < ntq; ++Q) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int rr = r0 + 8 * u, q = 32 * Q + rr, i = 32 * I + cc;
                if (q < d && i < d) tv[rr][cc] = q < k ? V[(long long)q * d + i] : make_double2(0.0, 0.0);
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int rr = r0 + 8 * u, i = 32 * I + rr, q = 32 * Q + cc;
                if (i < d && q < d) {
                    const d2 v = tv[cc][rr];
                    const double s = q < k ? sgn * (lam[q] - tau) : 0.0;
                    const long long e = (long long)i * d + q;
                    VT[e] = v;
                    P[e] = cscale(v, s);
                }
            }
            __syncthreads();
        }
    if (t == 0) a.st[b].C_z = a.lambda * base[a.hl.misc + 1];
}

// z = (Z + Z^H)/2 (prox_trace.m:146)
__global__ __launch_bounds__(256) void pl_take_z_kernel(PlArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    if (!a.act[b]) return;
    const int d = a.d;
    const long long o = (long long)b * d * d;
    const d2* Zn = reinterpret_cast<const d2*>(a.Znew) + o;
    d2* z = reinterpret_cast<d2*>(a.z) + o;
    // the prox's complement form (misc[2], trieig_kernel: more than half of the eigenvalues above tau): Zn holds
    // sum_{lam <= tau} (tau - lam) v v^H and z = Zn + (W + W^H)/2 - tau I, W = z_old - step G as pl_prox_in built it
    const double* mb = a.scratch + (long long)b * a.hl.stride + a.hl.misc;
    const bool side = mb[2] != 0.0;
    const double st = a.st[b].step, tau = a.tau[b];
    const d2* zo = reinterpret_cast<const d2*>(a.zo) + o;
    const d2* G = reinterpret_cast<const d2*>(a.G) + o;
    // by 32 x 32 tile pairs (I, J), (J, I) staged in LDS (as pl_prox_in_kernel): every entry read once, row-coalesced
    // (the element-wise form read Zn[j][i] down a column); the same expression per entry
    __shared__ d2 tu[32][33], tl[32][33], wu[32][33], wl[32][33];
    const int nt = (d + 31) / 32, cc = t & 31, r0 = t >> 5;
    for (int I = 0; I < nt; ++I)
        for (int J = I; J < nt; ++J) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rr = r0 + 8 * q;
                const int i1 = 32 * I + rr, j1 = 32 * J + cc, i2 = 32 * J + rr, j2 = 32 * I + cc;
                if (i1 < d && j1 < d) {
                    const long long e = (long long)i1 * d + j1;
                    tu[rr][cc] = Zn[e];
                    if (side) wu[rr][cc] = csub(zo[e], cscale(G[e], st));
                }
                if (i2 < d && j2 < d) {
                    const long long e = (long long)i2 * d + j2;
                    tl[rr][cc] = Zn[e];
                    if (side) wl[rr][cc] = csub(zo[e], cscale(G[e], st));
                }
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rr = r0 + 8 * q;
                const int i1 = 32 * I + rr, j1 = 32 * J + cc;
                if (i1 < d && j1 < d) {   // z[i1][j1] from u = Zn[i1][j1], l = Zn[j1][i1]
                    const d2 u = tu[rr][cc], l = tl[cc][rr];
                    d2 v = make_double2(0.5 * (u.x + l.x), 0.5 * (u.y - l.y));
                    if (side) {
                        const d2 w1 = wu[rr][cc], w2 = wl[cc][rr];
                        v = cadd(v, make_double2(0.5 * (w1.x + w2.x) - (i1 == j1 ? tau : 0.0), 0.5 * (w1.y - w2.y)));
                    }
                    z[(long long)i1 * d + j1] = v;
                }
                const int i2 = 32 * J + rr, j2 = 32 * I + cc;
                if (I != J && i2 < d && j2 < d) {
                    const d2 u = tl[rr][cc], l = tu[cc][rr];
                    d2 v = make_double2(0.5 * (u.x + l.x), 0.5 * (u.y - l.y));
                    if (side) {
                        const d2 w1 = wl[rr][cc], w2 = wu[cc][rr];
                        v = cadd(v, make_double2(0.5 * (w1.x + w2.x), 0.5 * (w1.y - w2.y)));
                    }
                    z[(long long)i2 * d + j2] = v;
                }
            }
            __syncthreads();
        }
}

// A(X) = diag(R^H X R) given T = X R: a_i = Re sum_r conj(R[r][i]) T[r][i]  (the imaginary part
// is rounding; initializeLinopPR.m:58 would carry it, and it cancels in every use)
__global__ __launch_bounds__(256) void pl_diagform_kernel(int d, int m, const double* Rp, const double* Tp,
                                                          double* out, const int* act) {
    const int b = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m || (act && !act[b])) return;
    const d2* R = reinterpret_cast<const d2*>(Rp);
    const d2* T = reinterpret_cast<const d2*>(Tp) + (long long)b * d * m;
    double s = 0.0;
    for (int r = 0; r < d; ++r) {
        const d2 rr = R[(long long)r * m + i], tt = T[(long long)r * m + i];
        s += rr.x * tt.x + rr.y * tt.y;
    }
    out[(long long)b * m + i] = s;
}

// tfocs_AT.m:55-71: x = z (theta = 1) or (1-theta) x_old + theta z, A_x by combination or
// recomputed when the counter fires; plus the reductions the backtracking and the stopping
// test need: ||x - y||^2, ||x||^2, <x - y, g_y>, ||x - x_old||^2.
__global__ __launch_bounds__(256) void pl_make_x_kernel(PlArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    __shared__ double red[16 * 4];
    PlState& p = a.st[b];
    if (!a.act[b]) return;
    const int d = a.d;
    const long long o = (long long)b * d * d;
    const d2* xo = reinterpret_cast<const d2*>(a.xo) + o;
    const d2* z = reinterpret_cast<const d2*>(a.z) + o;
    const d2* y = reinterpret_cast<const d2*>(a.y) + o;
    const d2* G = reinterpret_cast<const d2*>(a.G) + o;
    d2* x = reinterpret_cast<d2*>(a.x) + o;
    const bool one = !p.ycomp;
    const double th = p.theta, om = 1.0 - th;
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    for (long long e = t; e < (long long)d * d; e += 256) {
        const d2 xn = one ? z[e] : cadd(cscale(xo[e], om), cscale(z[e], th));
        x[e] = xn;
        const d2 xy = csub(xn, y[e]), dx = csub(xn, xo[e]);
        v[0] += cabs2(xy);
        v[1] += cabs2(xn);
        v[2] += xy.x * G[e].x + xy.y * G[e].y;
        v[3] += cabs2(dx);
    }
    block_sum<4>(v, red);
    __shared__ int need;
    if (t == 0) {
        p.xy_sq = v[0];
        p.nx2 = v[1];
        p.dot_xy_g = v[2];
        p.ndx2 = v[3];
        need = 0;
        if (one) {
            p.C_x = p.C_z;
        } else {
            if (p.cntr_Ax >= a.cntr_reset) {
                p.cntr_Ax = 0.0;
                need = 1;
            } else {
                p.cntr_Ax += 1.0;
            }
            p.C_x = INFINITY;
        }
        p.need_Ax = need;
        p.f_x = INFINITY;
        p.have_gAx = 0;
        if (need) atomicAdd(&a.cnt[2], 1);
    }
    __syncthreads();
    const long long ov = (long long)b * a.m;
    if (one) {
        for (int i = t; i < a.m; i += 256) a.Ax[ov + i] = a.Az[ov + i];
    } else if (!need) {
        for (int i = t; i < a.m; i += 256) a.Ax[ov + i] = om * a.Axo[ov + i] + th * a.Az[ov + i];
    }
}

__global__ __launch_bounds__(256) void pl_set_Ax_kernel(PlArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    if (!a.act[b] || !a.st[b].need_Ax) return;
    const long long o = (long long)b * a.m;
    for (int i = t; i < a.m; i += 256) a.Ax[o + i] = a.Aex[o + i];
}

// tfocs_backtrack.m: local Lipschitz estimate, leave the inner loop or grow L.
__global__ __launch_bounds__(256) void pl_backtrack_kernel(PlArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    __shared__ double red[16 * 2];
    PlState& p = a.st[b];
    if (!a.act[b]) return;
    const long long o = (long long)b * a.m;
    if (p.xy_sq == 0.0) {  // localL = Inf; do_break
        if (t == 0) {
            p.localL = INFINITY;
            p.inner = 0;
        }
        return;
    }
    const bool simple = p.backtrack_simple;
    // f_x (both branches need it; the non-simple one also g_Ax and <A_x - A_y, g_Ax - g_Ay>)
    double v[2] = {0.0, 0.0};
    for (int i = t; i < a.m; i += 256) {
        const double g = a.Ax[o + i] - a.bvec[o + i];
        v[0] += g * g;
        if (!simple) {
            a.gAx[o + i] = g;
            v[1] += (a.Ax[o + i] - a.Ay[o + i]) * (g - a.gAy[o + i]);
        }
    }
    block_sum<2>(v, red);
    if (t != 0) return;
    if (p.xy_sq / p.nx2 < 2.220446049250313e-16) p.cntr_Ax = INFINITY;  // force a reset
    double localL;
    if (simple) {
        p.f_x = 0.5 * v[0];
        const double q_x = p.f_y + p.dot_xy_g + 0.5 * p.L * p.xy_sq;
        localL = p.L + 2.0 * fmax(p.f_x - q_x, 0.0) / p.xy_sq;
        p.backtrack_simple = fabs(p.f_y - p.f_x) >= 1e-10 * fmax(fabs(p.f_x), fabs(p.f_y));
    } else {
        p.f_x = 0.5 * v[0];
        p.have_gAx = 1;
        localL = 2.0 * v[1] / p.xy_sq;
    }
    p.backtrack_steps += 1;
    p.localL = localL;
    if (localL <= p.L || p.L >= a.Lexact) {
        p.inner = 0;
        return;
    }
    double L = p.L;
    if (!isinf(localL)) L = fmin(a.Lexact, localL);
    else localL = L;
    p.L = fmin(a.Lexact, fmax(localL, L / a.beta));
}

// tfocs_iterate.m: stopping tests (stopCrit 1) and the periodic restart.
__global__ __launch_bounds__(256) void pl_iterate_kernel(PlArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    PlState& p = a.st[b];
    if (p.done) return;
    __shared__ int restart_now;
    if (t == 0) {
        p.n_iter += 1;
        const double norm_x = sqrt(p.nx2), norm_dx = sqrt(p.ndx2);
        int stop = 0;
        if (p.f_y != p.f_y) stop = 1;                                            // NaN found
        else if (norm_dx == 0.0) stop = p.n_iter > 1;                             // ||dx|| = 0
        else if (norm_dx < a.tol * fmax(norm_x, 1.0)) stop = 2;                   // step tolerance
        else if (p.n_iter == a.maxIts) stop = 3;                                  // iteration limit
        else if (p.backtrack_steps > 0 && p.xy_sq == 0.0) stop = 4;
        restart_now = 0;
        if (stop) {
            p.done = 1;
            p.status = stop;
            atomicAdd(&a.cnt[8], 1);
        } else {
            p.backtrack_steps = 0;
            if (p.n_iter - p.restart_iter == a.restart) {
                restart_now = 1;
                p.restart_iter = p.n_iter;
                p.backtrack_simple = 1;
                p.theta = INFINITY;
                p.f_y = p.f_x;
                p.have_gAy = p.have_gAx;
                p.have_gy = 0;
            }
        }
    }
    __syncthreads();
    if (!restart_now) return;
    // y = x, A_y = A_x, g_Ay = g_Ax, z = x, A_z = A_x
    const long long dd = 2LL * a.d * a.d, o = b * dd;
    for (long long e = t; e < dd; e += 256) {
        a.y[o + e] = a.x[o + e];
        a.z[o + e] = a.x[o + e];
    }
    const long long ov = (long long)b * a.m;
    for (int i = t; i < a.m; i += 256) {
        a.Ay[ov + i] = a.Ax[ov + i];
        a.Az[ov + i] = a.Ax[ov + i];
        a.gAy[ov + i] = a.gAx[ov + i];
    }
}

// ---- setup / output
// Upper Cholesky factor R of the Hermitian positive definite K (m x m): K = R^H R.
// One work-group; ok[0] = 0 on a non-positive pivot.
__global__ __launch_bounds__(256) void chol_kernel(int m, const double* Kp, double* Rp, int* ok) {
    const int t = threadIdx.x;
    const d2* K = reinterpret_cast<const d2*>(Kp);
    d2* R = reinterpret_cast<d2*>(Rp);
    __shared__ double piv;
    __shared__ int bad;
    if (t == 0) bad = 0;
    for (long long e = t; e < (long long)m * m; e += 256) R[e] = make_double2(0.0, 0.0);
    __syncthreads();
    for (int j = 0; j < m; ++j) {
        for (int i = j + t; i < m; i += 256) {
            d2 s = K[(long long)j * m + i];
            for (int k = 0; k < j; ++k) s = csub(s, cmulc(R[(long long)k * m + j], R[(long long)k * m + i]));
            R[(long long)j * m + i] = s;
        }
        __syncthreads();
        if (t == 0) {
            const double djj = R[(long long)j * m + j].x;
            if (!(djj > 0.0)) bad = 1;
            piv = sqrt(fmax(djj, 1e-300));
        }
        __syncthreads();
        const double inv = 1.0 / piv;
        for (int i = j + 1 + t; i < m; i += 256) R[(long long)j * m + i] = cscale(R[(long long)j * m + i], inv);
        if (t == 0) R[(long long)j * m + j] = make_double2(piv, 0.0);
        __syncthreads();
    }
    if (t == 0) ok[0] = !bad;
}

// dst[j][i] = src[i][j] (plain transpose, complex), rows x cols source
__global__ __launch_bounds__(256) void ztranspose_kernel(int rows, int cols, const double* Sp, double* Dp) {
    __shared__ d2 tile[32][33];
    const d2* S = reinterpret_cast<const d2*>(Sp);
    d2* D = reinterpret_cast<d2*>(Dp);
    const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int yy = ty; yy < 32; yy += 8) {
        const int r = r0 + yy, c = c0 + tx;
        if (r < rows && c < cols) tile[yy][tx] = S[(long long)r * cols + c];
    }
    __syncthreads();
    for (int yy = ty; yy < 32; yy += 8) {
        const int c = c0 + yy, r = r0 + tx;
        if (r < rows && c < cols) D[(long long)c * rows + r] = tile[tx][yy];
    }
}

// x (d x d) -> eigensolver matrix slot (the final eig, MyPhaseLift.m:106)
__global__ __launch_bounds__(256) void pl_final_in_kernel(int d, const double* xp, double* scratch, HeevLayout hl) {
    const int b = blockIdx.x;
    const d2* x = reinterpret_cast<const d2*>(xp) + (long long)b * d * d;
    d2* C = reinterpret_cast<d2*>(scratch + (long long)b * hl.stride + hl.C);
    for (long long e = threadIdx.x; e < (long long)d * d; e += 256) C[e] = x[e];
}

// sig_d = sqrt(lam_max) u; reduced coordinates: w = R^{-1} sig_d (back substitution, R upper),
// the n-space signal is then Phi^H w (GEMM by the host).
__global__ __launch_bounds__(256) void pl_final_vec_kernel(int d, int reduced, const double* Rp, const double* V1,
                                                           const double* scratch, HeevLayout hl, double* out) {
    const int b = blockIdx.x, t = threadIdx.x;
    extern __shared__ double smem[];
    d2* w = reinterpret_cast<d2*>(smem);
    const double lam = scratch[(long long)b * hl.stride + hl.lam];
    const d2* u = reinterpret_cast<const d2*>(V1) + (long long)b * d;
    // MATLAB: sqrt(eVal(end)) * V(:,end); X = Q Xd Q^H has n - d extra zero eigenvalues, so a
    // non-positive lam_max (Xd = 0) means the leading n-space eigenvalue is 0 and sig = 0.
    const double sl = reduced ? sqrt(fmax(lam, 0.0)) : sqrt(fabs(lam));
    const bool imag = !reduced && lam < 0.0;
    for (int i = t; i < d; i += 256) {
        const d2 v = cscale(u[i], sl);
        w[i] = imag ? make_double2(-v.y, v.x) : v;
    }
    __syncthreads();
    d2* o = reinterpret_cast<d2*>(out) + (long long)b * d;
    if (!reduced) {
        for (int i = t; i < d; i += 256) o[i] = w[i];
        return;
    }
    const d2* R = reinterpret_cast<const d2*>(Rp);
    __shared__ d2 wj;
    for (int j = d - 1; j >= 0; --j) {  // column-oriented back substitution
        if (t == 0) {
            const d2 rjj = R[(long long)j * d + j];
            const double inv = 1.0 / rjj.x;
            wj = cscale(w[j], inv);
            w[j] = wj;
        }
        __syncthreads();
        const d2 c = wj;
        for (int i = t; i < j; i += 256) w[i] = csub(w[i], cmul(R[(long long)i * d + j], c));
        __syncthreads();
    }
    for (int i = t; i < d; i += 256) o[i] = w[i];
}
// iterations and ACE_ST_* bits per realisation (stop 1/2: step tolerance reached)
__global__ __launch_bounds__(256) void pl_outputs_kernel(int batch, const PlState* st, int32_t* iters, uint32_t* status) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    if (iters) iters[b] = st[b].n_iter;
    if (status) status[b] |= (st[b].status == 1 || st[b].status == 2) ? ACE_ST_CONVERGED : 0u;
}
}  // namespace

void launch_pl_outputs(int batch, const PlState* st, int32_t* iters, uint32_t* status, hipStream_t s) {
    hipLaunchKernelGGL(pl_outputs_kernel, dim3((batch + 255) / 256), dim3(256), 0, s, batch, st, iters, status);
}
void launch_pl_init(const PlArgs& a, hipStream_t st) { hipLaunchKernelGGL(pl_init_kernel, dim3(a.batch), dim3(256), 0, st, a); }
void launch_pl_outer_begin(const PlArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(pl_outer_begin_kernel, dim3(a.batch), dim3(256), 0, st, a);
}
void launch_pl_theta(const PlArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(pl_theta_kernel, dim3((a.batch + 255) / 256), dim3(256), 0, st, a);
}
void launch_pl_make_y(const PlArgs& a, hipStream_t st) { hipLaunchKernelGGL(pl_make_y_kernel, dim3(a.batch), dim3(256), 0, st, a); }
void launch_pl_set_Ay(const PlArgs& a, hipStream_t st) { hipLaunchKernelGGL(pl_set_Ay_kernel, dim3(a.batch), dim3(256), 0, st, a); }
void launch_pl_grad(const PlArgs& a, hipStream_t st) { hipLaunchKernelGGL(pl_grad_kernel, dim3(a.batch), dim3(256), 0, st, a); }
void launch_pl_prox_in(const PlArgs& a, hipStream_t st) { hipLaunchKernelGGL(pl_prox_in_kernel, dim3(a.batch), dim3(256), 0, st, a); }
void launch_pl_assemble(const PlArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(pl_assemble_kernel, dim3(a.batch), dim3(256), 0, st, a);
}
void launch_pl_take_z(const PlArgs& a, hipStream_t st) { hipLaunchKernelGGL(pl_take_z_kernel, dim3(a.batch), dim3(256), 0, st, a); }
void launch_pl_make_x(const PlArgs& a, hipStream_t st) { hipLaunchKernelGGL(pl_make_x_kernel, dim3(a.batch), dim3(256), 0, st, a); }
void launch_pl_set_Ax(const PlArgs& a, hipStream_t st) { hipLaunchKernelGGL(pl_set_Ax_kernel, dim3(a.batch), dim3(256), 0, st, a); }
void launch_pl_backtrack(const PlArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(pl_backtrack_kernel, dim3(a.batch), dim3(256), 0, st, a);
}
void launch_pl_iterate(const PlArgs& a, hipStream_t st) { hipLaunchKernelGGL(pl_iterate_kernel, dim3(a.batch), dim3(256), 0, st, a); }
void launch_pl_diagform(int d, int m, int batch, const double* R, const double* T, double* out, const int* act,
                        hipStream_t st) {
    hipLaunchKernelGGL(pl_diagform_kernel, dim3((m + 255) / 256, batch), dim3(256), 0, st, d, m, R, T, out, act);
}
void launch_chol(int m, const double* K, double* R, int* ok, hipStream_t st) {
    hipLaunchKernelGGL(chol_kernel, dim3(1), dim3(256), 0, st, m, K, R, ok);
}
void launch_ztranspose(int rows, int cols, const double* S, double* D, hipStream_t st) {
    dim3 grid((cols + 31) / 32, (rows + 31) / 32);
    hipLaunchKernelGGL(ztranspose_kernel, grid, dim3(256), 0, st, rows, cols, S, D);
}
void launch_pl_final_in(int d, int batch, const double* x, double* scratch, HeevLayout hl, hipStream_t st) {
    hipLaunchKernelGGL(pl_final_in_kernel, dim3(batch), dim3(256), 0, st, d, x, scratch, hl);
}
void launch_pl_final_vec(int d, int batch, int reduced, const double* R, const double* V1, const double* scratch,
                         HeevLayout hl, double* out, hipStream_t st) {
    hipLaunchKernelGGL(pl_final_vec_kernel, dim3(batch), dim3(256), 16 * (size_t)d, st, d, reduced, R, V1, scratch,
                       hl, out);
}

}  // namespace ace
