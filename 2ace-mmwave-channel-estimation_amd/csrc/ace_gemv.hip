// Private-codebook regime (one A per realisation) and setup kernels.
//
// With a private A every iteration streams the realisation's own matrices
// (A twice, G and K once) from HBM, so these kernels are HBM-bound GEMVs:
// rows are read as contiguous 16-B complex128 per lane (1 KiB per wave
// instruction), the per-realisation vector sits in LDS, and wave64 shuffles
// finish each row's dot product.  The conjugate-transpose product A^H g also
// streams A row-major: each thread owns output columns and walks the rows, so
// A never needs a transposed copy.
#include "ace_common.hpp"

#include <algorithm>

namespace ace {

namespace {
constexpr int ROWS_PER_WG = 32;  // 8 rows per wave, 4 at a time

template <int MODE>
__global__ __launch_bounds__(256) void zgemv_rows_kernel(int M, int K, const double* __restrict__ L,
                                                         long long strideL, const double* __restrict__ V, int ldv,
                                                         double* __restrict__ C, const double* __restrict__ E,
                                                         int ldc) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    d2* vs = reinterpret_cast<d2*>(smem);
    const int b = blockIdx.x;
    const d2* Vb = reinterpret_cast<const d2*>(V) + (long long)b * ldv;
    for (int k = threadIdx.x; k < K; k += blockDim.x) vs[k] = Vb[k];
    __syncthreads();
    const d2* Lb = reinterpret_cast<const d2*>(L) + (long long)b * strideL;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int rbase = blockIdx.y * ROWS_PER_WG + w * 8;
    for (int g = 0; g < 2; ++g) {
        const int r0 = rbase + g * 4;
        d2 acc[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = make_double2(0.0, 0.0);
        for (int k = lane; k < K; k += 64) {
            const d2 v = vs[k];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = r0 + q;
                if (r < M) {
                    const d2 a = Lb[(long long)r * K + k];
                    acc[q].x += a.x * v.x - a.y * v.y;
                    acc[q].y += a.x * v.y + a.y * v.x;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            acc[q].x = wave_sum(acc[q].x);
            acc[q].y = wave_sum(acc[q].y);
        }
        if (lane < 4) {
            const int r = r0 + lane;
            d2 s = acc[0];
            if (lane == 1) s = acc[1];
            if (lane == 2) s = acc[2];
            if (lane == 3) s = acc[3];
            if (r < M) {
                d2* out = reinterpret_cast<d2*>(C) + (long long)b * ldc + r;
                if (MODE == 1) s = csub(reinterpret_cast<const d2*>(E)[(long long)b * ldc + r], s);
                else if (MODE == 2) s = cadd(reinterpret_cast<const d2*>(E)[(long long)b * ldc + r], s);
                *out = s;
            }
        }
    }
}

// C[b][k] = epi( sum_i conj(L_b[i][k]) V[b][i] )
template <int MODE>
__global__ __launch_bounds__(256) void zgemv_cols_kernel(int M, int K, const double* __restrict__ L,
                                                         long long strideL, const double* __restrict__ V, int ldv,
                                                         double* __restrict__ C, const double* __restrict__ E,
                                                         int ldc) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    d2* vs = reinterpret_cast<d2*>(smem);
    const int b = blockIdx.x;
    const d2* Vb = reinterpret_cast<const d2*>(V) + (long long)b * ldv;
    for (int i = threadIdx.x; i < M; i += blockDim.x) vs[i] = Vb[i];
    __syncthreads();
    const int k = blockIdx.y * blockDim.x + threadIdx.x;
    if (k >= K) return;
    const d2* Lb = reinterpret_cast<const d2*>(L) + (long long)b * strideL + k;
    d2 acc0 = make_double2(0.0, 0.0), acc1 = acc0;
    int i = 0;
    for (; i + 8 <= M; i += 8) {
        d2 a[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) a[q] = Lb[(long long)(i + q) * K];
#pragma unroll
        for (int q = 0; q < 8; q += 2) {
            const d2 v0 = vs[i + q], v1 = vs[i + q + 1];
            acc0.x += a[q].x * v0.x + a[q].y * v0.y;
            acc0.y += a[q].x * v0.y - a[q].y * v0.x;
            acc1.x += a[q + 1].x * v1.x + a[q + 1].y * v1.y;
            acc1.y += a[q + 1].x * v1.y - a[q + 1].y * v1.x;
        }
    }
    for (; i < M; ++i) {
        const d2 a = Lb[(long long)i * K], v = vs[i];
        acc0.x += a.x * v.x + a.y * v.y;
        acc0.y += a.x * v.y - a.y * v.x;
    }
    d2 s = cadd(acc0, acc1);
    const long long off = (long long)b * ldc + k;
    if (MODE == 1) s = csub(reinterpret_cast<const d2*>(E)[off], s);
    else if (MODE == 2) s = cadd(reinterpret_cast<const d2*>(E)[off], s);
    reinterpret_cast<d2*>(C)[off] = s;
}

// In-place Gauss-Jordan inverse of (I + K), K Hermitian PSD => I + K HPD, no pivoting.
// One 1024-thread work-group per matrix; G holds K on entry, (I+K)^{-1} on exit.
__global__ __launch_bounds__(1024) void inv_ipk_kernel(int m, double* __restrict__ Gall, long long strideG) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    d2* rowk = reinterpret_cast<d2*>(smem);
    d2* colk = rowk + m;
    d2* G = reinterpret_cast<d2*>(Gall) + (long long)blockIdx.x * strideG;
    const int t = threadIdx.x, nt = blockDim.x;
    for (int i = t; i < m; i += nt) G[(long long)i * m + i].x += 1.0;
    __syncthreads();
    for (int k = 0; k < m; ++k) {
        const d2 p = G[(long long)k * m + k];
        const double den = p.x * p.x + p.y * p.y;
        const d2 pinv = make_double2(p.x / den, -p.y / den);
        for (int j = t; j < m; j += nt) {
            const d2 a = (j == k) ? make_double2(1.0, 0.0) : G[(long long)k * m + j];
            rowk[j] = cmul(a, pinv);
            colk[j] = (j == k) ? make_double2(0.0, 0.0) : G[(long long)j * m + k];
        }
        __syncthreads();
        for (int e = t; e < m * m; e += nt) {
            const int i = e / m, j = e - i * m;
            d2* gij = &G[(long long)i * m + j];
            if (i == k) {
                *gij = rowk[j];
            } else {
                const d2 base = (j == k) ? make_double2(0.0, 0.0) : *gij;
                *gij = csub(base, cmul(colk[i], rowk[j]));
            }
        }
        __syncthreads();
    }
}
// max |x_i| over the grid: per-block maxima combined with a 64-bit atomic max on the bit patterns
// (for non-negative doubles the unsigned order of the patterns is the numeric order); *out must be
// zeroed first (launch_max_abs does it).  A NaN entry yields +inf.
__global__ __launch_bounds__(256) void max_abs_kernel(long long n, const double* __restrict__ x, double* out) {
    __shared__ double part[256];
    double v = 0.0;
    // (a NaN counts as +inf: fmax would drop it, and callers use the maximum as a convergence test)
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += 256LL * gridDim.x) {
        const double a = fabs(x[i]);
        v = fmax(v, a == a ? a : INFINITY);
    }
    part[threadIdx.x] = v;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) part[threadIdx.x] = fmax(part[threadIdx.x], part[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0)
        atomicMax(reinterpret_cast<unsigned long long*>(out), (unsigned long long)__double_as_longlong(part[0]));
}
// Newton-Schulz start for the HPD matrix I + K, one row per block: Ap = I + K, Id = I, and the
// Gershgorin bound b = max_i sum_j |(I + K)_ij| into *bnd (atomic max; zeroed first).
__global__ __launch_bounds__(256) void ns_rows_kernel(int m, const d2* __restrict__ K, d2* __restrict__ Ap,
                                                      d2* __restrict__ Id, double* bnd) {
    __shared__ double part[256];
    const int i = blockIdx.x;
    double rs = 0.0;
    for (int j = threadIdx.x; j < m; j += 256) {
        d2 v = K[(long long)i * m + j];
        if (i == j) v.x += 1.0;
        rs += sqrt(v.x * v.x + v.y * v.y);
        Ap[(long long)i * m + j] = v;
        Id[(long long)i * m + j] = make_double2(i == j ? 1.0 : 0.0, 0.0);
    }
    part[threadIdx.x] = rs;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMax(reinterpret_cast<unsigned long long*>(bnd), (unsigned long long)__double_as_longlong(part[0]));
}
__global__ __launch_bounds__(256) void ns_x0_kernel(int m, const double* __restrict__ bnd, d2* __restrict__ X0) {
    const long long e = blockIdx.x * 256LL + threadIdx.x;
    if (e >= (long long)m * m) return;
    const double alpha = 2.0 / (1.0 + *bnd);
    X0[e] = make_double2((e / m) == (e % m) ? alpha : 0.0, 0.0);
}
}  // namespace

void launch_ns_prep(int m, const double* K, double* Ap, double* Id, double* X0, hipStream_t st, double* bnd) {
    (void)hipMemsetAsync(bnd, 0, sizeof(double), st);
    hipLaunchKernelGGL(ns_rows_kernel, dim3(m), dim3(256), 0, st, m, (const d2*)K, (d2*)Ap, (d2*)Id, bnd);
    hipLaunchKernelGGL(ns_x0_kernel, dim3((unsigned)(((long long)m * m + 255) / 256)), dim3(256), 0, st, m, bnd, (d2*)X0);
}

void launch_max_abs(long long n, const double* x, double* out, hipStream_t st) {
    (void)hipMemsetAsync(out, 0, sizeof(double), st);
    const long long blocks = std::min<long long>(1024, (n + 2047) / 2048);
    hipLaunchKernelGGL(max_abs_kernel, dim3((unsigned)std::max<long long>(1, blocks)), dim3(256), 0, st, n, x, out);
}

__global__ __launch_bounds__(256) void hermitize_kernel(int m, d2* __restrict__ X) {
    const int j = blockIdx.x * 16 + (threadIdx.x & 15), i = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (i >= m || j >= m || j < i) return;
    const d2 u = X[(long long)i * m + j];
    if (i == j) {
        X[(long long)i * m + j] = make_double2(u.x, 0.0);
        return;
    }
    const d2 l = X[(long long)j * m + i];
    const d2 h = make_double2(0.5 * (u.x + l.x), 0.5 * (u.y - l.y));
    X[(long long)i * m + j] = h;
    X[(long long)j * m + i] = make_double2(h.x, -h.y);
}
void launch_hermitize(int m, double* X, hipStream_t st) {
    const dim3 grid((m + 15) / 16, (m + 15) / 16);
    hipLaunchKernelGGL(hermitize_kernel, grid, dim3(256), 0, st, m, reinterpret_cast<d2*>(X));
}

void launch_zgemv_rows(int mode, int M, int K, int nb, const double* L, long long strideL, const double* V,
                       int ldv, double* C, const double* E, int ldc, hipStream_t st) {
    dim3 grid(nb, (M + ROWS_PER_WG - 1) / ROWS_PER_WG), block(256);
    const size_t sh = (size_t)K * sizeof(d2);
    if (mode == 0) hipLaunchKernelGGL(zgemv_rows_kernel<0>, grid, block, sh, st, M, K, L, strideL, V, ldv, C, E, ldc);
    else if (mode == 1) hipLaunchKernelGGL(zgemv_rows_kernel<1>, grid, block, sh, st, M, K, L, strideL, V, ldv, C, E, ldc);
    else hipLaunchKernelGGL(zgemv_rows_kernel<2>, grid, block, sh, st, M, K, L, strideL, V, ldv, C, E, ldc);
}

void launch_zgemv_cols(int mode, int M, int K, int nb, const double* L, long long strideL, const double* V,
                       int ldv, double* C, const double* E, int ldc, hipStream_t st) {
    dim3 grid(nb, (K + 255) / 256), block(256);
    const size_t sh = (size_t)M * sizeof(d2);
    if (mode == 0) hipLaunchKernelGGL(zgemv_cols_kernel<0>, grid, block, sh, st, M, K, L, strideL, V, ldv, C, E, ldc);
    else if (mode == 1) hipLaunchKernelGGL(zgemv_cols_kernel<1>, grid, block, sh, st, M, K, L, strideL, V, ldv, C, E, ldc);
    else hipLaunchKernelGGL(zgemv_cols_kernel<2>, grid, block, sh, st, M, K, L, strideL, V, ldv, C, E, ldc);
}

void launch_inv_ipk(int m, int count, double* G, long long strideG, hipStream_t st) {
    hipLaunchKernelGGL(inv_ipk_kernel, dim3(count), dim3(1024), (size_t)2 * m * sizeof(d2), st, m, G, strideG);
}

}  // namespace ace
