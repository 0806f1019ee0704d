// Microbenchmark of the look-ahead dense-tail factorisation (developer tool,
// not part of the library): an nt x nt well-conditioned quasi-definite lower
// triangle (dfl001's widened tail is nt = 4441) factored by the library's
// k_tail_pr steps, one HIP event pair per step; the pivots are checked
// against a host LDL' (nt <= 2048) and, built with -DIPO_PANEL_STAMPS, the
// in-kernel clock stamps of workgroup 0 of one step are printed.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off [-DIPO_PANEL_STAMPS] \
//         -I linear-programming-vanderbei_amd/csrc tools/ubench_tail.hip -o tools/ubench_tail
//   tools/ubench_tail [nt] [reps] [stamp step]
#include "../linear-programming-vanderbei_amd/csrc/kkt_dense.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

int main(int argc, char** argv) {
    const int nt = argc > 1 ? std::atoi(argv[1]) : 4441;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const int ntb = (nt + 63) / 64;
    const int stamp_step = argc > 3 ? std::atoi(argv[3]) : ntb - 8;
    std::mt19937_64 rng(1);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    // K = [-E A; A' D]-like signs on the diagonal, dominant so that no pivot is near zero
    std::vector<double> S((size_t)nt * nt, 0.0), dsc(nt);
    for (int c = 0; c < nt; c++)
        for (int r = c; r < nt; r++) S[r + (size_t)c * nt] = r == c ? (c & 1 ? -1.0 : 1.0) * (0.2 * nt + 1.0) : 0.1 * U(rng);
    for (int c = 0; c < nt; c++) dsc[c] = std::fabs(S[c + (size_t)c * nt]);
    std::vector<int> sign(nt);
    for (int c = 0; c < nt; c++) sign[c] = c & 1 ? -1 : 1;
    double *dS, *dS0, *dW, *ddg, *ddsc, *ddsc0;
    int *dlive, *dflags, *dsign;
    const size_t bytes = (size_t)nt * nt * sizeof(double);
    CK(hipMalloc(&dS, bytes)); CK(hipMalloc(&dS0, bytes)); CK(hipMalloc(&dW, (size_t)ntb * nt * 64 * 8));
    CK(hipMalloc(&ddg, nt * 8)); CK(hipMalloc(&ddsc, nt * 8)); CK(hipMalloc(&ddsc0, nt * 8));
    CK(hipMalloc(&dlive, nt * 4)); CK(hipMalloc(&dflags, 16)); CK(hipMalloc(&dsign, nt * 4));
    CK(hipMemcpy(dS0, S.data(), bytes, hipMemcpyHostToDevice));
    CK(hipMemcpy(ddsc0, dsc.data(), nt * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsign, sign.data(), nt * 4, hipMemcpyHostToDevice));
    ipo::PlanView pv{};
    pv.dg = ddg; pv.live = dlive; pv.flags = dflags; pv.sign = dsign; pv.dscale = ddsc; pv.tau = 1e-17;
    ipo::TailView tv{};
    tv.S = dS; tv.nt = nt; tv.ntb = ntb; tv.tc = 0; tv.W = dW;
    if (const char* vb = std::getenv("IPO_HIP_VISIT_BLOCKS")) tv.vk = std::atoi(vb);
    // the library's visit schedule (IPO_HIP_VISIT_SCHED=0: the visit_hi formula alone)
    std::vector<int> vptr;
    unsigned* dvl = nullptr;
    const char* vs = std::getenv("IPO_HIP_VISIT_SCHED");
    if (!vs || std::atoi(vs) != 0) {
        int cus = 0;
        CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
        const std::vector<unsigned> vl = ipo::tail_visit_schedule(ntb, nt, tv.vk, cus, vptr);
        CK(hipMalloc(&dvl, vl.size() * sizeof(unsigned) + 4));
        CK(hipMemcpy(dvl, vl.data(), vl.size() * sizeof(unsigned), hipMemcpyHostToDevice));
        tv.vlist = dvl;
        tv.vptr = vptr.data();
        std::printf("visit schedule on %d CUs: workgroups per launch", cus);
        for (int t = 0; t < ntb; t++) std::printf(" %d", std::max(1, (nt - t * 64 + 63) / 64 - 1) + vptr[t + 1] - vptr[t]);
        std::printf("\n");
    }
    // the persistent run (UB_RUN=1, k_tail_run, latest chunk UB_LATEST blocks):
    // timed as one launch, its pivots and factor compared with the per-step
    // launches' (another grouping of the visits' sums: not bitwise)
    // UB_WINPUB=0: the run without the window hand-off (RunPub)
    // UB_CHAIN=1: the chain launch (k_tail_chain_run) instead of the run
    const bool chain = std::getenv("UB_CHAIN") && std::atoi(std::getenv("UB_CHAIN")) != 0;
    const bool run = chain || (std::getenv("UB_RUN") && std::atoi(std::getenv("UB_RUN")) != 0);
    std::vector<int> rptr;
    uint2* ditems = nullptr;
    int* dcnt = nullptr;
    double *dpub = nullptr, *dsave = nullptr;
    int ub_latest = 0;
    int cus_run = 0;
    if (run) {
        CK(hipDeviceGetAttribute(&cus_run, hipDeviceAttributeMultiprocessorCount, 0));
        if (const char* cp = std::getenv("UB_CAP")) cus_run = std::atoi(cp);   // the schedule's items per launch
        const int latest = std::getenv("UB_LATEST") ? std::atoi(std::getenv("UB_LATEST")) : ipo::kTailVisitLatest;
        const std::vector<uint2> items = chain ? ipo::tail_chain_schedule(ntb, nt, tv.vk, latest, cus_run, rptr)
                                               : ipo::tail_run_schedule(ntb, nt, tv.vk, latest, cus_run, rptr);
        if (chain) rptr[ntb] = static_cast<int>(items.size());
        if (chain && std::getenv("UB_NOVISIT")) {      // timing of the chain and tile items alone (factor wrong)
            std::vector<uint2> kept;
            for (const uint2& it : items)
                if (it.y >> 30) kept.push_back(it);
            const_cast<std::vector<uint2>&>(items) = kept;
            rptr[ntb] = static_cast<int>(kept.size());
        }
        ub_latest = latest;
        CK(hipMalloc(&ditems, items.size() * sizeof(uint2)));
        CK(hipMemcpy(ditems, items.data(), items.size() * sizeof(uint2), hipMemcpyHostToDevice));
        CK(hipMalloc(&dcnt, ipo::chain_zero_ints(ntb) * sizeof(int)));
        CK(hipMalloc(&dpub, (size_t)ntb * 4 * ipo::kChainWinPub * sizeof(double)));
        CK(hipMalloc(&dsave, (2 * 64 * 64 + 64) * sizeof(double)));
        std::printf("persistent run: %zu items, latest chunk %d, items per launch", items.size(), latest);
        for (int t = 0; t < ntb; t++) std::printf(" %d", rptr[t + 1] - rptr[t]);
        std::printf("\n");
    }
    // UB_TRACE=file: the last timed run's per-item trace (k_tail_run's
    // {drawn, ready, done, xcc}, 100 MHz ticks) with each item's record, binary
    unsigned long long* dtrace = nullptr;
    const char* trace_file = std::getenv("UB_TRACE");
    const size_t trace_n = (size_t)(rptr.empty() ? 0 : rptr[ntb] + ntb) * 4 + (size_t)ntb * 32;
    if (run && trace_file) CK(hipMalloc(&dtrace, trace_n * sizeof(unsigned long long)));
    double* dwpub = nullptr;
    int* dwflag = nullptr;
    int wepoch = 0;
    if (run && !chain && !(std::getenv("UB_WINPUB") && std::atoi(std::getenv("UB_WINPUB")) == 0)) {
        CK(hipMalloc(&dwpub, 2 * (size_t)ntb * 4 * ipo::kTailPubWin * sizeof(double)));
        CK(hipMalloc(&dwflag, (size_t)ntb * ntb * 4 * sizeof(int)));
        CK(hipMemset(dwflag, 0, (size_t)ntb * ntb * 4 * sizeof(int)));
        std::printf("window hand-off on\n");
    }
    auto run_once = [&](hipStream_t st) {
        CK(hipMemsetAsync(dcnt, 0, ipo::chain_zero_ints(ntb) * sizeof(int), st));
        if (chain) {
            ipo::ChainRun rc;
            rc.items = ditems;
            rc.n = rptr[ntb];
            rc.ticket = dcnt;
            rc.abort = dcnt + 1;
            rc.pdone = dcnt + 2;
            rc.rdone = rc.pdone + ntb;
            rc.vseq = rc.rdone + ntb * ntb;
            rc.dwin = rc.vseq + ntb * ntb;
            rc.dpub = dpub;
            rc.save = dsave;
            rc.latest = ub_latest;
            rc.novisit = std::getenv("UB_NOVISIT") ? 1 : 0;
            rc.trace = dtrace;
            ipo::launch_tail_chain(pv, tv, rc, st);
        } else {
            ipo::TailRun rc;
            rc.items = ditems;
            rc.n = rptr[ntb];
            rc.t0 = 0;
            rc.ticket = dcnt;
            rc.pdone = dcnt + 1;
            rc.vseq = dcnt + 1 + ntb;
            if (dwpub) {          // the window hand-off (UB_WINPUB=0: off), as the library's default
                rc.pub = dwpub;
                rc.wflag = dwflag;
                rc.pread = dcnt + 1 + ntb + ntb * ntb;
                rc.epoch = ++wepoch;
            }
            rc.trace = dtrace;
            ipo::launch_tail_run(pv, tv, rc, st);
        }
    };
    std::vector<double> g_step;
    if (run) {      // the per-step launches' pivots and factor, for the comparison
        CK(hipMemcpy(dS, dS0, bytes, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(ddsc, ddsc0, nt * 8, hipMemcpyDeviceToDevice));
        CK(hipMemset(dflags, 0, 16));
        for (int t = 0; t < ntb; t++) ipo::launch_tail_step(pv, tv, t, 0);
        CK(hipDeviceSynchronize());
        g_step.resize(nt);
        CK(hipMemcpy(g_step.data(), ddg, nt * 8, hipMemcpyDeviceToHost));
    }
    std::vector<hipEvent_t> ev(ntb + 1);
    for (auto& e : ev) CK(hipEventCreate(&e));
    std::vector<double> step_us(ntb, 0.0);
    double total = 0.0;
    const size_t wst = (size_t)nt * 64;
    for (int r = 0; r < reps + 1; r++) {
        CK(hipMemcpy(dS, dS0, bytes, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(ddsc, ddsc0, nt * 8, hipMemcpyDeviceToDevice));
        CK(hipMemset(dflags, 0, 16));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(ev[0], 0));
        if (run) {
            run_once(0);
            CK(hipEventRecord(ev[ntb], 0));
        } else {
            for (int t = 0; t < ntb; t++) {
                ipo::launch_tail_step(pv, tv, t, 0);
                CK(hipEventRecord(ev[t + 1], 0));
            }
        }
        CK(hipEventSynchronize(ev[ntb]));
        if (r == 0) continue;       // warm-up
        float ms = 0;
        CK(hipEventElapsedTime(&ms, ev[0], ev[ntb]));
        total += ms;
        for (int t = 0; t < ntb && !run; t++) {
            CK(hipEventElapsedTime(&ms, ev[t], ev[t + 1]));
            step_us[t] += 1e3 * ms;
        }
    }
    int fl[4];
    CK(hipMemcpy(fl, dflags, 16, hipMemcpyDeviceToHost));
    const double flops = (double)nt * nt * nt / 3.0;
    std::printf("visit chunk %d; ", tv.vk);
    std::printf("nt %d (%d block columns): %.3f ms per factor, %.2f TFLOP/s of nt^3/3, bail flags %d %d %d\n", nt, ntb,
                total / reps, flops / (total / reps * 1e-3) / 1e12, fl[0], fl[1], fl[2]);
    std::printf("per step (us):");
    for (int t = 0; t < ntb; t++) std::printf("%s%.1f", t % 16 ? " " : "\n  ", step_us[t] / reps);
    std::printf("\n");
    if (run) {
        std::vector<double> g(nt);
        CK(hipMemcpy(g.data(), ddg, nt * 8, hipMemcpyDeviceToHost));
        double mx = 0;
        int same = 0;
        for (int k = 0; k < nt; k++) {
            mx = std::fmax(mx, std::fabs(g[k] - g_step[k]) / std::fabs(g_step[k]));
            same += g[k] == g_step[k];
        }
        std::printf("persistent run vs per-step launches: pivots max relative difference %.2e, %d of %d bitwise\n", mx,
                    same, nt);
        if (dtrace) {
            const size_t ni = rptr[ntb];
            std::vector<unsigned long long> tr(chain ? trace_n : ni * 4);
            std::vector<uint2> items(ni);
            CK(hipMemcpy(tr.data(), dtrace, tr.size() * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(items.data(), ditems, ni * sizeof(uint2), hipMemcpyDeviceToHost));
            FILE* f = std::fopen(trace_file, "wb");
            const int hdr[2] = {ntb, (int)ni * (chain ? -1 : 1)};
            std::fwrite(hdr, 4, 2, f);
            std::fwrite(items.data(), sizeof(uint2), ni, f);
            std::fwrite(tr.data(), 8, tr.size(), f);
            std::fclose(f);
        }
    }
    if (nt <= 2048) {       // host LDL' (right-looking, the reference form l = a / d, a -= l (l_c d))
        std::vector<double> A = S, d(nt);
        for (int k = 0; k < nt; k++) {
            const double dk = A[k + (size_t)k * nt];
            d[k] = dk;
            for (int i = k + 1; i < nt; i++) A[i + (size_t)k * nt] /= dk;
            for (int j = k + 1; j < nt; j++) {
                const double c = A[j + (size_t)k * nt] * dk;
                for (int i = j; i < nt; i++) A[i + (size_t)j * nt] -= A[i + (size_t)k * nt] * c;
            }
        }
        std::vector<double> g(nt);
        CK(hipMemcpy(g.data(), ddg, nt * 8, hipMemcpyDeviceToHost));
        double mx = 0;
        for (int k = 0; k < nt; k++) mx = std::fmax(mx, std::fabs(g[k] - d[k]) / std::fabs(d[k]));
        std::printf("pivots vs host LDL': max relative difference %.2e\n", mx);
    }
#ifdef IPO_PANEL_STAMPS
    // one more run up to the stamped step, so the stamps are that step's
    CK(hipMemcpy(dS, dS0, bytes, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(ddsc, ddsc0, nt * 8, hipMemcpyDeviceToDevice));
    CK(hipMemset(dflags, 0, 16));
    for (int t = 0; t <= stamp_step; t++) ipo::launch_tail_step(pv, tv, t, 0);
    CK(hipDeviceSynchronize());
    long long st[8][16];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(ipo::g_stamps), sizeof(st)));
    std::printf("step %d, workgroup 0 stamps (cycles since wave 0 entry); slots: 15 entry, 3 pre-update operands in LDS, "
                "4 products formed, 14 pre-update done, 0 loaded, 6 last column of the previous window seen, 7 its update applied, "
                "1 after updates, 5 own last column published, 2 window done, 12 end, 13 done\n",
                stamp_step);
    const long long b = st[0][15];
    for (int w = 0; w < 8; w++) {
        std::printf("wave %d:", w);
        for (int sl : {15, 3, 4, 14, 0, 6, 7, 1, 5, 2, 12, 13}) std::printf(" %d:%lld", sl, st[w][sl] - b);
        std::printf("\n");
    }
#endif
    return 0;
}
