/*
 * oracle/oracle_cli.c — TEST INFRASTRUCTURE ONLY.
 * Command-line front end of the oracle (used by tests/ and bench.py's cpu_baseline).
 *   edsbwt_oracle transform <file.eds> <base>        EDS-BWTransform.sh:1-31 (naive GSA)
 *   edsbwt_oracle search <base> <patterns> [a] [threads] [limit]
 *       MOVE_EDSBWTSearch <base> <patterns> (mainMove_EDSBWT.cpp:17-62): writes
 *       <patterns>output_M_LF.csv, prints "bs took:<secs>" on stdout and
 *       count_found / count_not_found on stderr (MOVE_EDSBWTSearch.cpp:145,154-155).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "edsbwt_oracle.h"

int main(int argc, char** argv) {
    if (argc >= 4 && !strcmp(argv[1], "transform")) {
        if (orc_transform(argv[2], argv[3])) { fprintf(stderr, "%s\n", orc_last_error()); return 1; }
        fprintf(stderr, "File %s done.\n", argv[2]);
        return 0;
    }
    if (argc >= 4 && !strcmp(argv[1], "search")) {
        unsigned a = argc > 4 ? (unsigned)atoi(argv[4]) : 8;
        int threads = argc > 5 ? atoi(argv[5]) : 1;
        unsigned long long limit = argc > 6 ? strtoull(argv[6], 0, 10) : 0;
        orc_engine* E = orc_open(argv[2], a, 0);
        if (!E) { fprintf(stderr, "%s\n", orc_last_error()); return 1; }
        char* out = malloc(strlen(argv[3]) + 32);
        sprintf(out, "%soutput_M_LF.csv", argv[3]);
        orc_counters c;
        double secs = 0;
        if (orc_search_file(E, argv[3], out, limit, threads, &c, &secs)) { fprintf(stderr, "%s\n", orc_last_error()); return 1; }
        printf("bs took:%g", secs);
        fflush(stdout);
        fprintf(stderr, "\ncount_found = %llu\ncount_not_found = %llu\n", (unsigned long long)c.found, (unsigned long long)c.not_found);
        fprintf(stderr, "interval_steps = %llu\nstep_moves = %llu\nlocate_moves = %llu\npdf_calls = %llu\neof_reads = %llu\noccurrences = %llu\nr_prime = %u\nruns = %u\n",
                (unsigned long long)c.interval_steps, (unsigned long long)c.step_moves, (unsigned long long)c.locate_moves,
                (unsigned long long)c.pdf_calls, (unsigned long long)c.eof_reads, (unsigned long long)c.occurrences,
                orc_r_prime(E), orc_runs(E));
        orc_close(E);
        free(out);
        return 1; /* mainMove_EDSBWT.cpp:61 returns 1 on success */
    }
    fprintf(stderr, "usage: %s transform <file.eds> <base> | search <base> <patterns> [a] [threads] [limit]\n", argv[0]);
    return 2;
}
