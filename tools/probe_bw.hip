// Probe: achievable HBM bandwidth on gfx950 (read-only reduction, write-only fill, copy),
// 16-byte accesses, grid-stride, 1 GiB footprint.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef double d2v __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void rd(const d2v* __restrict__ a, long long n, double* out) {
    d2v s = {0.0, 0.0};
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256 * 4) {
        d2v v0 = a[i], v1 = i + gridDim.x * 256LL < n ? a[i + gridDim.x * 256LL] : d2v{0, 0};
        d2v v2 = i + 2 * gridDim.x * 256LL < n ? a[i + 2 * gridDim.x * 256LL] : d2v{0, 0};
        d2v v3 = i + 3 * gridDim.x * 256LL < n ? a[i + 3 * gridDim.x * 256LL] : d2v{0, 0};
        s += v0 + v1 + v2 + v3;
    }
    if (s.x == 1234.5) out[0] = s.y;
}
__global__ __launch_bounds__(256) void wr(d2v* __restrict__ a, long long n) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) a[i] = d2v{1.0, 2.0};
}
__global__ __launch_bounds__(256) void cp(const d2v* __restrict__ a, d2v* __restrict__ b, long long n) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) b[i] = a[i];
}

int main() {
    const long long bytes = 1LL << 30, n = bytes / 16;
    d2v *a, *b;
    double* o;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&o, 8));
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int grid : {1024, 2048, 4096, 8192}) {
        for (int k = 0; k < 3; ++k) {
            for (int w = 0; w < 2; ++w) {   // warm-up, then timed
                CK(hipEventRecord(e0));
                const int R = w ? 10 : 1;
                for (int r = 0; r < R; ++r) {
                    if (k == 0) rd<<<grid, 256>>>(a, n, o);
                    else if (k == 1) wr<<<grid, 256>>>(b, n);
                    else cp<<<grid, 256>>>(a, b, n);
                }
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (w) printf("grid %5d %s: %.2f TB/s\n", grid, k == 0 ? "read " : (k == 1 ? "write" : "copy "),
                              (k == 2 ? 2.0 : 1.0) * bytes * R / (ms * 1e-3) / 1e12);
            }
        }
    }
    return 0;
}
