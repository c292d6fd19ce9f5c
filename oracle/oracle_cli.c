/*
 * ORACLE (test infrastructure only) -- command line front end of the C
 * restatement: `gsc_oracle <in.wav> <out.gsc> [encoder.lpr options]
 * [--threads=N] [--stats]`.  Options follow encoder.lpr:1957-1998.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "gsc_oracle.h"

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s <in.wav> <out.gsc> [-cs8 -cpf4096 ...] [--threads=N] [--stats]\n", argv[0]);
        return 2;
    }
    int threads = 1, stats = 0;
    const char *opts[64];
    int no = 0;
    for (int i = 3; i < argc && no < 64; i++) {
        if (strncmp(argv[i], "--threads=", 10) == 0) threads = atoi(argv[i] + 10);
        else if (strcmp(argv[i], "--stats") == 0) stats = 1;
        else opts[no++] = argv[i];
    }
    gsc_params p;
    ora_default_params(&p);
    ora_parse_params(&p, no, opts);
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 1; }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char *wav = (unsigned char *)malloc((size_t)n);
    if (fread(wav, 1, (size_t)n, f) != (size_t)n) { fclose(f); return 1; }
    fclose(f);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    uint8_t *out = NULL;
    size_t out_len = 0;
    int rc = ora_encode(wav, (size_t)n, &p, threads, &out, &out_len);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (rc != 0) { fprintf(stderr, "encode failed: %d\n", rc); return 1; }
    FILE *o = fopen(argv[2], "wb");
    fwrite(out, 1, out_len, o);
    fclose(o);
    if (stats) {
        ora_stats s;
        ora_get_stats(&s);
        double sec = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
        printf("{\"bytes\": %zu, \"seconds\": %.3f, \"frames\": %d, \"scan_iterations\": %lld, "
               "\"kd_searches\": %lld, \"kd_leaves\": %lld, \"kd_splits\": %lld}\n",
               out_len, sec, s.frame_count, s.scan_iterations, s.kd_searches, s.kd_leaves, s.kd_splits);
    }
    ora_free(out);
    free(wav);
    return 0;
}
