/*
 * orc_cli.c -- ORACLE command line (test infrastructure only, see orc.h).
 * Usage: ipo_oracle file.mps [hsd|intpt|hsdls]
 * Prints exactly what the reference `ipo file.mps` prints (main.c:16-58,
 * minus the .out file), so the output can be diffed against the captured
 * traces in tests/golden/netlib/<name>.mps.sol.  Timing goes to stderr.
 */
#include <stdio.h>
#include <string.h>
#include "orc.h"

int main(int argc, char **argv)
{
    if (argc < 2) { fprintf(stderr, "usage: %s file.mps [hsd|intpt|hsdls]\n", argv[0]); return 1; }
    int method = 0;
    if (argc > 2 && !strcmp(argv[2], "intpt")) method = 1;
    if (argc > 2 && !strcmp(argv[2], "hsdls")) method = 2;
    orc_run run; memset(&run, 0, sizeof(run));
    int st = orc_ipo_run(argv[1], method, stdout, &run);
    fprintf(stderr, "oracle: status=%d iters=%d setup=%.3fs total=%.3fs it/s=%.3f\n",
            st, run.iters, run.t_setup, run.t_total,
            run.iters > 0 && run.t_total > 0 ? run.iters / run.t_total : 0.0);
    return st < 0 ? 1 : 0;
}
