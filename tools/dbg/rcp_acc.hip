// Accuracy of the raw v_rcp_f64 seed against the IEEE reciprocal over random doubles (development probe).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdint>
__global__ void k(const double* x, long long* ulp, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double r = __builtin_amdgcn_rcp(x[i]);
    const double e = 1.0 / x[i];
    long long a = __double_as_longlong(r), b = __double_as_longlong(e);
    ulp[i] = a > b ? a - b : b - a;
}
int main() {
    const int n = 1 << 22;
    double* h = (double*)malloc(8 * (size_t)n);
    uint64_t s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const double m = 1.0 + (double)(s >> 11) / 9007199254740992.0;
        const int ex = (int)((s >> 3) % 200) - 100;
        h[i] = ((s & 1) ? -1.0 : 1.0) * ldexp(m, ex);
    }
    double* dx; long long* du;
    hipMalloc(&dx, 8 * (size_t)n); hipMalloc(&du, 8 * (size_t)n);
    hipMemcpy(dx, h, 8 * (size_t)n, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, du, n);
    long long* hu = (long long*)malloc(8 * (size_t)n);
    hipMemcpy(hu, du, 8 * (size_t)n, hipMemcpyDeviceToHost);
    long long mx = 0, cnt[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; ++i) { mx = hu[i] > mx ? hu[i] : mx; cnt[hu[i] < 3 ? hu[i] : 3]++; }
    printf("v_rcp_f64 vs 1/x: max %lld ulp; 0 ulp %lld, 1 ulp %lld, 2 ulp %lld, >2 ulp %lld of %d\n", mx, cnt[0], cnt[1], cnt[2], cnt[3], n);
    return 0;
}
