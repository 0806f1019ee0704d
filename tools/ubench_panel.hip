// Microbenchmark of the fused panel kernels on a synthetic dense tail
// (developer tool, not part of the library): nt x nt well-conditioned
// quasi-definite lower triangle, block column kb = 0 (the widest launch),
// k_panel (kind 1) vs k_panel_w (kind 2), plus the in-kernel clock stamps
// of k_panel_w's workgroup 0.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -DIPO_PANEL_STAMPS \
//         -I linear-programming-vanderbei_amd/csrc tools/ubench_panel.hip -o tools/ubench_panel
#include "../linear-programming-vanderbei_amd/csrc/kkt_dense.hip"

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

int main(int argc, char** argv) {
    const int nt = argc > 1 ? std::atoi(argv[1]) : 2766;
    const int kb = argc > 2 ? std::atoi(argv[2]) : 0;
    const int reps = 20;
    std::mt19937_64 rng(1);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    std::vector<double> S((size_t)nt * nt, 0.0), dsc(nt), sgn(nt);
    for (int c = 0; c < nt; c++)
        for (int r = c; r < nt; r++) S[r + (size_t)c * nt] = r == c ? (c & 1 ? -1.0 : 1.0) * (nt + 1.0) : 0.1 * U(rng);
    for (int c = 0; c < nt; c++) dsc[c] = std::fabs(S[c + (size_t)c * nt]);
    std::vector<int> sign(nt);
    for (int c = 0; c < nt; c++) sign[c] = c & 1 ? -1 : 1;
    double *dS, *dS0, *dW, *ddg, *ddsc;
    int *dlive, *dflags, *dsign;
    const size_t bytes = (size_t)nt * nt * sizeof(double);
    CK(hipMalloc(&dS, bytes)); CK(hipMalloc(&dS0, bytes)); CK(hipMalloc(&dW, bytes));
    CK(hipMalloc(&ddg, nt * 8)); CK(hipMalloc(&ddsc, nt * 8));
    CK(hipMalloc(&dlive, nt * 4)); CK(hipMalloc(&dflags, 16)); CK(hipMalloc(&dsign, nt * 4));
    CK(hipMemcpy(dS0, S.data(), bytes, hipMemcpyHostToDevice));
    CK(hipMemcpy(ddsc, dsc.data(), nt * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsign, sign.data(), nt * 4, hipMemcpyHostToDevice));
    ipo::PlanView pv{};
    pv.dg = ddg; pv.live = dlive; pv.flags = dflags; pv.sign = dsign; pv.dscale = ddsc; pv.tau = 1e-17;
    ipo::TailView tv{};
    tv.S = dS; tv.nt = nt; tv.ntb = (nt + 63) / 64; tv.tc = 0; tv.W = dW;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<double> out[3];
    for (int kind : {1, 2}) {
        ipo::g_panel_kind = kind;
        float tot = 0;
        for (int r = 0; r < reps + 2; r++) {
            CK(hipMemcpy(dS, dS0, bytes, hipMemcpyDeviceToDevice));
            CK(hipMemset(dflags, 0, 16));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            ipo::launch_panel(pv, nullptr, nullptr, 0, 0, tv, kb, 0);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) tot += ms;
        }
        int fl[2];
        CK(hipMemcpy(fl, dflags, 8, hipMemcpyDeviceToHost));
        out[kind].resize((size_t)nt * nt);
        CK(hipMemcpy(out[kind].data(), dS, bytes, hipMemcpyDeviceToHost));
        std::printf("kind %d: %.2f us per launch (nt %d, kb %d, bail %d)\n", kind, 1e3 * tot / reps, nt, kb, fl[1]);
    }
    if (kb > 0) {   // look-ahead step kb: panel kb (with block kb - 1's pre-update) beside R(kb - 1)
        double* dW2;
        CK(hipMalloc(&dW2, (size_t)nt * 64 * 8));
        CK(hipMemset(dW2, 0, (size_t)nt * 64 * 8));
        float tot = 0;
        for (int r = 0; r < reps + 2; r++) {
            CK(hipMemcpy(dS, dS0, bytes, hipMemcpyDeviceToDevice));
            CK(hipMemset(dflags, 0, 16));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            ipo::launch_tail_step(pv, tv, kb, dW2, dW, 0);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) tot += ms;
        }
        std::printf("tail step %d: %.2f us per launch\n", kb, 1e3 * tot / reps);
    }
    size_t diff = 0;
    for (size_t i = 0; i < out[1].size(); i++) diff += out[1][i] != out[2][i];
    std::printf("entries differing between kinds: %zu\n", diff);
#ifdef IPO_PANEL_STAMPS
    long long st[8][16];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(ipo::g_stamps), sizeof(st)));
    std::printf("k_panel_w workgroup 0 stamps (cycles since wave 0 entry); slots: 15 entry, 3 pre-update operands in LDS, 4 products formed, 14 pre-update done, 0 loaded, 1 after updates, 2 window done, 12 end, 13 done\n");
    const long long b = st[0][15];
    for (int w = 0; w < 8; w++) {
        std::printf("wave %d:", w);
        for (int sl : {15, 3, 4, 14, 0, 1, 2, 12, 13}) std::printf(" %d:%lld", sl, st[w][sl] - b);
        std::printf("\n");
    }
#endif
    return 0;
}
