// ipo_main.cpp -- `ipo_hip file.mps [hsd|intpt|hsdls]`: the reference's ipo driver
// (src/common/main.c:16-58) on top of libipo_hip.so; same stdout, no .out file.
// Extra timing goes to stderr so stdout can be diffed against .sol traces.
#include <cstdio>
#include <cstring>

#include "../../include/ipo_hip.h"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s file.mps [hsd|intpt|hsdls]\n", argv[0]);
        return 1;
    }
    int method = 0;
    if (argc > 2 && !std::strcmp(argv[2], "intpt")) method = 1;
    if (argc > 2 && !std::strcmp(argv[2], "hsdls")) method = 2;
    ipo_hip_stats st;
    const int status = ipo_hip_run_mps(argv[1], method, stdout, 1, &st);
    std::fprintf(stderr,
                 "ipo_hip: status=%d iters=%d setup=%.3fs solve=%.3fs it/s=%.2f factor=%.1fms solve=%.1fms "
                 "lnz=%ld nsup=%d levels=%d\n",
                 status, st.iters, st.t_setup_s, st.t_solve_s, st.iters > 0 ? st.iters / st.t_solve_s : 0.0,
                 st.factor_ms, st.solve_ms, st.lnz, st.nsup, st.nlevels);
    return status < 0 ? 1 : 0;
}
