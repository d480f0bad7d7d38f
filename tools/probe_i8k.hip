// Probe: time the int8 digit-plane applies (ace_i8gemm.hip) in isolation at the unit's
// shape (batch 4096, m = 256, n = 1024), built in variants that drop one resource at a
// time (-DACE_I8_PROBE_NO_LDS: A fragments from registers; -DACE_I8_PROBE_NO_B: codebook
// fragments from registers).  Diagnostic only.
#include "../2ace-mmwave-channel-estimation_amd/csrc/ace_i8gemm.hip"
#include <cstdio>
#include <vector>
#include <random>
using namespace ace;
#define CK(x) do { hipError_t e_ = (x); if (e_) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
int main() {
    const int nb = 4096, m = 256, n = 1024;
    std::vector<double> A(2 * m * n);
    std::mt19937_64 r(1);
    for (int i = 0; i < m * n; ++i) {
        const int c = r() & 3;
        A[2 * i] = (c == 0) - (c == 2);
        A[2 * i + 1] = (c == 1) - (c == 3);
    }
    double *dA, *c8, *Z, *N, *Y, *M, *T, *g, *W;
    int8_t *LA, *LH;
    int* flag;
    RealState* rs;
    CK(hipMalloc(&dA, A.size() * 8));
    CK(hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&c8, 8));
    double one = 1.0;
    CK(hipMemcpy(c8, &one, 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&LA, i8_frag_bytes(m, n)));
    CK(hipMalloc(&LH, i8_frag_bytes(n, m)));
    CK(hipMemset(LA, 0, i8_frag_bytes(m, n)));
    CK(hipMemset(LH, 0, i8_frag_bytes(n, m)));
    CK(hipMalloc(&flag, 4));
    CK(hipMemset(flag, 0, 4));
    launch_i8_expand(m, n, dA, c8, LA, LH, flag, 0);
    const size_t bn = (size_t)nb * n * 16, bm = (size_t)nb * m * 16;
    CK(hipMalloc(&Z, bn)); CK(hipMalloc(&N, bn)); CK(hipMalloc(&W, bn));
    CK(hipMalloc(&Y, bm)); CK(hipMalloc(&M, bm)); CK(hipMalloc(&T, bm)); CK(hipMalloc(&g, bm));
    CK(hipMemset(Z, 0, bn)); CK(hipMemset(N, 0, bn)); CK(hipMemset(Y, 0, bm)); CK(hipMemset(M, 0, bm));
    CK(hipMemset(g, 0, bm));
    std::vector<RealState> hs(nb);
    for (auto& s : hs) { s = RealState{}; s.mu = 1.0; s.vbound = 1.0; }
    CK(hipMalloc(&rs, nb * sizeof(RealState)));
    CK(hipMemcpy(rs, hs.data(), nb * sizeof(RealState), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int which = 0; which < 2; ++which) {
        auto run = [&]() {
            if (which == 0) launch_i8_apply_A(nb, n, m, LA, Z, N, Y, M, T, c8, rs, N, nullptr, 0);
            else launch_i8_apply_AH(nb, m, n, LH, g, W, c8, rs, 0);
        };
        for (int i = 0; i < 3; ++i) run();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        const int R = 20;
        for (int i = 0; i < R; ++i) run();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double macs = (double)nb * 8 * 2 * m * 2 * n;
        printf("%s: %.1f us/launch, %.0f int8 TOPS\n", which ? "apply_AH" : "apply_A", 1e3 * ms / R,
               2 * macs / (ms / R * 1e-3) / 1e12);
    }
    return 0;
}
