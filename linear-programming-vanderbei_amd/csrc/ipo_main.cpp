// ipo_main.cpp -- `ipo_hip file.mps [hsd|intpt|hsdls] [--free=split] [--no-out]`:
// the reference's ipo driver (src/common/main.c:16-58) on top of
// libipo_hip.so; same stdout, and like main.c:54-56 the solution report
// <NAME>.out (iolp.c:976-1045) in the working directory unless --no-out.
// --free=split: the free-variable extension (include/ipo_hip.h).  Extra
// timing goes to stderr so stdout can be diffed against .sol traces.
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/ipo_hip.h"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s file.mps [hsd|intpt|hsdls] [--free=split] [--no-out]\n", argv[0]);
        return 1;
    }
    int method = 0, flags = 0;
    bool out = true;
    for (int a = 2; a < argc; a++) {
        if (!std::strcmp(argv[a], "intpt")) method = 1;
        else if (!std::strcmp(argv[a], "hsdls")) method = 2;
        else if (!std::strcmp(argv[a], "--free=split")) flags |= IPO_HIP_SPLIT_FREE;
        else if (!std::strcmp(argv[a], "--no-out")) out = false;
    }
    std::string solfile;
    if (out) {
        // main.c:57-58: the NAME card's name, truncated, + ".out"
        FILE* f = std::fopen(argv[1], "r");
        char line[256], w0[256] = "", w1[256] = "";
        while (f && std::fgets(line, sizeof line, f)) {
            if (line[0] == '*') continue;
            if (std::sscanf(line, "%255s%255s", w0, w1) >= 1 && !std::strncmp(w0, "NAME", 4)) {
                solfile = std::string(w1).substr(0, 123) + ".out";
                break;
            }
        }
        if (f) std::fclose(f);
    }
    ipo_hip_stats st;
    std::memset(&st, 0, sizeof st);          // a run that stops before the solve fills none of it
    const int status = ipo_hip_run_mps_ex(argv[1], method, flags, solfile.empty() ? nullptr : solfile.c_str(), stdout,
                                          1, &st);
    std::fprintf(stderr,
                 "ipo_hip: status=%d iters=%d setup=%.3fs solve=%.3fs it/s=%.2f factor=%.1fms solve=%.1fms "
                 "lnz=%ld nsup=%d levels=%d\n",
                 status, st.iters, st.t_setup_s, st.t_solve_s, st.iters > 0 ? st.iters / st.t_solve_s : 0.0,
                 st.factor_ms, st.solve_ms, st.lnz, st.nsup, st.nlevels);
    return status < 0 ? 1 : 0;
}
