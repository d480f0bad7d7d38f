// Probe: time gyk_kernel (ace_i8gemm.hip) in isolation at the unit's shape (batch 4096,
// m = 256), in variants -DACE_GYK_PROBE_ONLY_A (g = G T only) / -DACE_GYK_PROBE_NO_C
// (without K Y).  Diagnostic only.
#include "../2ace-mmwave-channel-estimation_amd/csrc/ace_i8gemm.hip"
#include <cstdio>
#include <vector>
using namespace ace;
#define CK(x) do { hipError_t e_ = (x); if (e_) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
int main() {
    const int nb = 4096, m = 256;
    const size_t bm = (size_t)nb * m * 16;
    double *G, *Gf, *T, *B, *Yo, *M, *Yn, *g, *KYo, *KYn, *oY, *c8;
    int8_t* LK;
    RealState* rs;
    CK(hipMalloc(&G, (size_t)m * m * 16));
    CK(hipMalloc(&Gf, gyk_gfrag_bytes(m)));
    for (double** p : {&T, &Yo, &M, &Yn, &g, &KYo, &KYn, &oY}) { CK(hipMalloc(p, bm)); CK(hipMemset(*p, 0, bm)); }
    CK(hipMalloc(&B, bm / 2));
    CK(hipMemset(B, 0, bm / 2));
    CK(hipMemset(G, 0, (size_t)m * m * 16));
    CK(hipMalloc(&LK, i8k_frag_bytes(m)));
    CK(hipMemset(LK, 1, i8k_frag_bytes(m)));
    CK(hipMalloc(&c8, 16));
    double c2[2] = {1.0, 1.0};
    CK(hipMemcpy(c8, c2, 16, hipMemcpyHostToDevice));
    std::vector<RealState> hs(nb);
    for (auto& s : hs) { s = RealState{}; s.mu = 1.0; s.opt_obj = 1e300; }
    CK(hipMalloc(&rs, nb * sizeof(RealState)));
    CK(hipMemcpy(rs, hs.data(), nb * sizeof(RealState), hipMemcpyHostToDevice));
    launch_gyk_gfrag(m, G, Gf, 0);
    const GykArgs a{Gf, T, B, Yo, M, Yn, g, KYo, KYn, oY, LK, c8, rs};
    for (int i = 0; i < 3; ++i) launch_gyk(nb, m, a, 0);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int i = 0; i < 20; ++i) launch_gyk(nb, m, a, 0);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("gyk: %.1f us/launch (f64 G T at 3M: %.1f TF/s)\n", 1e3 * ms / 20, 6.0 * nb * m * m / (ms / 20 * 1e-3) / 1e12);
    return 0;
}
