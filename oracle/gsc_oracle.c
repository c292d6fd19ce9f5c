/*
 * ORACLE (test infrastructure only) -- SoundChunks encoder restated in C.
 * Every function cites the reference encoder/encoder.lpr lines it follows.
 * Build: oracle/Makefile (-O2 -ffp-contract=off, no fast-math).
 */
#include "gsc_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include "ann_oracle.h"
#include "fpc_rtl.h"
#include "yakmo_oracle.h"

#define C_MAX_ATTENUATION 15
#define C_MAX_CHUNKS_PER_FRAME 4096
#define MAX_SINGLE 3.4028234663852886e+38 /* MaxSingle as Double */

static ora_stats g_stats;
static pthread_mutex_t g_stats_mu = PTHREAD_MUTEX_INITIALIZER;

void ora_free(void *p) { free(p); }
void ora_get_stats(ora_stats *s) { *s = g_stats; }

/* ---- parameters (encoder.lpr:201-227, 1486-1509, 1983-1998) ------------- */
void ora_default_params(gsc_params *p) {
    memset(p, 0, sizeof(*p));
    p->bit_rate = -1;
    p->precision = 3;
    p->low_cut = 0.0;
    p->high_cut = 24000.0;
    p->chunk_bit_depth = 8;
    p->chunk_size = 4;
    p->chunks_per_frame = C_MAX_CHUNKS_PER_FRAME;
    p->reduce_bass_band = 1;
    p->vfr = 1.0;
    p->chunk_blend = 0;
    p->frame_length = 4000.0;
}

static int param_start(int argc, const char *const *argv, const char *pfx) {
    size_t l = strlen(pfx);
    for (int i = 0; i < argc; i++)
        if (strncmp(argv[i], pfx, l) == 0) return i;
    return -1;
}
static int has_param(int argc, const char *const *argv, const char *p) {
    for (int i = 0; i < argc; i++)
        if (strcasecmp(argv[i], p) == 0) return 1;
    return 0;
}
static double param_value(int argc, const char *const *argv, const char *pfx, double def) {
    int i = param_start(argc, argv, pfx);
    if (i < 0) return def;
    const char *s = argv[i] + strlen(pfx);
    char *end = NULL;
    if (!*s) return def;
    double v = strtod(s, &end);
    if (!end || *end) return def; /* StrToFloatDef */
    return v;
}
static double clampd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }
static long long clampll(long long v, long long lo, long long hi) { return v < lo ? lo : (v > hi ? hi : v); }

void ora_parse_params(gsc_params *p, int argc, const char *const *argv) {
    p->bit_rate = (int)fpc_round(param_value(argc, argv, "-br", p->bit_rate));
    p->precision = (int)fpc_round(param_value(argc, argv, "-pr", p->precision));
    p->low_cut = param_value(argc, argv, "-lc", p->low_cut);
    p->high_cut = param_value(argc, argv, "-hc", p->high_cut);
    p->vfr = clampd(param_value(argc, argv, "-vfr", p->vfr), 0.0, 1.0);
    {
        double fl = param_value(argc, argv, "-fl", p->frame_length);
        p->frame_length = fl > 1.0 ? fl : 1.0;
    }
    p->chunk_bit_depth = (int)clampll(fpc_round(param_value(argc, argv, "-cbd", p->chunk_bit_depth)), 1, 16);
    p->chunk_size = (int)fpc_round(param_value(argc, argv, "-cs", p->chunk_size));
    p->chunks_per_frame =
        (int)clampll(fpc_round(param_value(argc, argv, "-cpf", p->chunks_per_frame)), 256, C_MAX_CHUNKS_PER_FRAME);
    p->verbose = has_param(argc, argv, "-v");
    p->reduce_bass_band = !has_param(argc, argv, "-pbb");
    p->chunk_blend = (int)clampll(fpc_round(param_value(argc, argv, "-cb", p->chunk_blend)), 0, p->chunk_size / 2);
    p->python_reduce = has_param(argc, argv, "-py");
}

/* ---- quantisers (encoder.lpr:1648-1698) ---------------------------------- */
int16_t ora_make_output_sample(double smp, int bd, int atten, int neg, double law) {
    double coeff = 1.0;
    for (int i = 0; i <= atten; i++) coeff += (double)i * law;
    int obd = (1 << (bd - 1)) - 1;
    long long r = fpc_round(smp * (double)obd * coeff);
    int16_t s16 = (int16_t)r;
    if (neg) s16 = (int16_t)(-(int)s16);
    int v = s16;
    if (v < -obd + 1) v = -obd + 1;
    if (v > obd - 1) v = obd - 1;
    return (int16_t)v;
}

double ora_make_float_sample(int16_t smp, int bd, int atten, int neg, double law) {
    double coeff = 1.0;
    for (int i = 0; i <= atten; i++) coeff += (double)i * law;
    double obd = (double)((1 << (bd - 1)) - 1);
    int16_t s16 = smp;
    if (neg) s16 = (int16_t)(-(int)s16);
    double r = (double)s16 / (obd * coeff);
    if (r < -1.0) r = -1.0;
    if (r > 1.0) r = 1.0;
    return r;
}

int ora_compute_attenuation(int cs, const double *samples, double law) {
    long long hi = 0;
    for (int i = 0; i < cs; i++) {
        long long c = fpc_ceil(fabs(samples[i] * 32767.0));
        if (c > hi) hi = c;
    }
    int r = 0;
    double coeff = 1.0;
    do {
        r++;
        coeff += (double)r * law;
    } while (!(((double)hi * coeff > 32767.0) || (r > C_MAX_ATTENUATION)));
    return r - 1;
}

/* TChunk.ComputeDstAttributes (encoder.lpr:365-397) */
static void dst_attributes(int cs, const double *src, double law, int *atten, int *neg, int *rev) {
    *atten = ora_compute_attenuation(cs, src, law);
    double p1 = 0.0, p2 = 0.0;
    for (int i = 0; i < cs; i++)
        if (src[i] < 0) p1 -= src[i];
    for (int i = 0; i < cs; i++)
        if (src[i] > 0) p2 += src[i];
    *neg = p1 > p2;
    p1 = 0.0;
    p2 = 0.0;
    for (int i = 0; i < cs / 2; i++) p1 += fabs(src[i]);
    for (int i = cs / 2; i < cs; i++) p2 += fabs(src[i]);
    *rev = p1 > p2;
}

/* ---- trig tables (exact FPC values; argument sets are finite) ----------- */
typedef struct {
    int cs;
    double *dct_cos;             /* [k*cs+n] cos(((pi/cs)*(n+0.5))*k) */
    double *dft_cos, *dft_sin;   /* [k*cs+i] of ((-2pi*k)*i)/cs */
    double *idft_cos, *idft_sin; /* [k*cs+i] of ((2pi*k)*i)/cs */
} trig_t;

static trig_t *g_trig[257];
static pthread_mutex_t g_trig_mu = PTHREAD_MUTEX_INITIALIZER;

static const trig_t *get_trig(int cs) {
    pthread_mutex_lock(&g_trig_mu);
    trig_t *t = g_trig[cs];
    if (!t) {
        t = (trig_t *)calloc(1, sizeof(trig_t));
        t->cs = cs;
        size_t n2 = (size_t)cs * cs;
        t->dct_cos = (double *)malloc(8 * n2);
        t->dft_cos = (double *)malloc(8 * n2);
        t->dft_sin = (double *)malloc(8 * n2);
        t->idft_cos = (double *)malloc(8 * n2);
        t->idft_sin = (double *)malloc(8 * n2);
        const double PI = 3.14159265358979323846;
        for (int k = 0; k < cs; k++)
            for (int n = 0; n < cs; n++) {
                t->dct_cos[k * cs + n] = fpc_cos(PI / (double)cs * ((double)n + 0.5) * (double)k);
                double a = ((-2.0 * PI) * (double)k) * (double)n / (double)cs;
                t->dft_cos[k * cs + n] = fpc_cos(a);
                t->dft_sin[k * cs + n] = fpc_sin(a);
                double b = ((2.0 * PI) * (double)k) * (double)n / (double)cs;
                t->idft_cos[k * cs + n] = fpc_cos(b);
                t->idft_sin[k * cs + n] = fpc_sin(b);
            }
        g_trig[cs] = t;
    }
    pthread_mutex_unlock(&g_trig_mu);
    return t;
}

/* TChunk.ComputeDCT + TEncoder.ComputeDCT + cepstrum (encoder.lpr:258-322,349-363,1700-1716) */
void ora_chunk_features(int cs, const double *src, int neg, int rev, double *dct) {
    const trig_t *t = get_trig(cs);
    double data[256], temp[256];
    for (int i = 0; i < cs; i++) data[i] = src[rev ? cs - 1 - i : i] * (neg ? -1.0 : 1.0);
    const double sqrt_half = sqrt(0.5), norm = sqrt(2.0 / (double)cs);
    for (int k = 0; k < cs; k++) {
        double s = (k == 0) ? sqrt_half : 1.0;
        double sum = 0;
        for (int n = 0; n < cs; n++) sum += s * data[n] * t->dct_cos[k * cs + n];
        dct[k] = sum * norm;
    }
    /* DFT */
    for (int k = 0; k < cs; k++) {
        double re = 0, im = 0;
        for (int i = 0; i < cs; i++) {
            re += data[i] * t->dft_cos[k * cs + i];
            im += data[i] * t->dft_sin[k * cs + i];
        }
        temp[k] = re * re + im * im;
    }
    for (int i = 0; i < cs; i++)
        if (!fpc_iszero(temp[i])) temp[i] = fpc_log10(temp[i]);
    /* iDFT(wave=data, frequencies=temp) */
    for (int k = 0; k < cs; k++) {
        double re = 0, im = 0;
        for (int i = 0; i < cs; i++) {
            re += temp[i] * t->idft_cos[k * cs + i];
            im += temp[i] * t->idft_sin[k * cs + i];
        }
        re /= (double)cs;
        im /= (double)cs;
        data[k] = sqrt(re * re + im * im);
    }
    for (int i = 0; i < cs; i++) dct[i + cs] = data[i] * 0.00001;
}

/* ---- FindAttenuationDivider (encoder.lpr:566-605) ----------------------- */
int ora_find_atten_divider(const double *src, int channels, long stride, int sample_count, int cs, int bd) {
    int best_div = 1;
    double best = MAX_SINGLE;
    double tmp[256];
    for (int i = 1; i <= 64; i++) {
        double law = 1.0 / (double)i;
        double v = 0;
        for (int j = 0; j < channels; j++)
            for (int k = 0; k < sample_count / cs; k++) {
                const double *p = src + (long)j * stride + (long)k * cs;
                for (int l = 0; l < cs; l++) tmp[l] = p[l];
                int atten = ora_compute_attenuation(cs, tmp, law);
                for (int l = 0; l < cs; l++) {
                    int16_t os = ora_make_output_sample(tmp[l], bd, atten, 0, law);
                    double fs = ora_make_float_sample(os, bd, atten, 0, law);
                    double d = tmp[l] - fs;
                    v += d * d;
                }
            }
        if (v < best) {
            best = v;
            best_div = i;
        }
    }
    return best_div;
}

/* ---- FPC TFPSList.QuickSort (encoder.exe @0x10003d410), count desc ------- */
static void qsort_fpc(int *items, const int *counts, int L, int R) {
    int I, J, P;
    do {
        I = L;
        J = R;
        P = (L + R) >> 1;
        do {
            int piv = counts[items[P]];
            /* Compare(piv, item) = CompareValue(item.Count, piv.Count) */
            while (counts[items[I]] > piv) I++;
            while (counts[items[J]] < piv) J--;
            if (I <= J) {
                int tmp = items[I];
                items[I] = items[J];
                items[J] = tmp;
                if (P == I) P = J;
                else if (P == J) P = I;
                I++;
                J--;
            }
        } while (I <= J);
        if (L < J) qsort_fpc(items, counts, L, J);
        L = I;
    } while (I < R);
}

void ora_sort_count_desc(int n, const int *counts, int *perm) {
    for (int i = 0; i < n; i++) perm[i] = i;
    if (n > 1) qsort_fpc(perm, counts, 0, n - 1);
}

/* ---- KNNScanReduce (encoder.lpr:699-765) -------------------------------- */
int ora_scan_reduce_n(int N, int D, const float *X, int K, float *C, int *clusters, int precision, int max_passes) {
    float **rows = (float **)malloc(sizeof(float *) * (size_t)K);
    for (int j = 0; j < K; j++) rows[j] = C + (size_t)j * D;
    int *cnts[2];
    cnts[0] = (int *)malloc(sizeof(int) * (size_t)K);
    cnts[1] = (int *)malloc(sizeof(int) * (size_t)K);
    for (int j = 0; j < K; j++) cnts[0][j] = cnts[1][j] = 1;
    int iter = 0;
    double err = MAX_SINGLE, prev_err;
    double tol = 1.0;
    for (int i = 0; i < precision; i++) tol *= 10.0; /* IntPower(10,-p) = 1/10^p */
    tol = 1.0 / tol;
    long long leaves = 0, splits = 0;
    for (;;) {
        prev_err = err;
        err = 0;
        ora_kdtree *kdt = ora_kdtree_create(rows, K, D, 1);
        int odd = iter & 1;
        for (int i = 0; i < N; i++) {
            float best;
            int b = ora_kdtree_search(kdt, X + (size_t)i * D, 0.0f, &best);
            long lv, sp;
            ora_kdtree_last_stats(kdt, &lv, &sp);
            leaves += lv;
            splits += sp;
            float rate = (float)(1.0 / sqrt((double)cnts[!odd][b]));
            float *c = C + (size_t)b * D;
            const float *x = X + (size_t)i * D;
            for (int k = 0; k < D; k++) {
                float v = x[k] - c[k];
                c[k] = c[k] + v * rate;
            }
            clusters[i] = b;
            err += (double)sqrtf(best / (float)D);
            cnts[odd][b] += 1;
        }
        for (int j = 0; j < K; j++) cnts[!odd][j] = 1;
        iter++;
        ora_kdtree_destroy(kdt);
        double diff = err > prev_err ? err - prev_err : prev_err - err;
        if (diff <= tol || iter >= max_passes) break;
    }
    pthread_mutex_lock(&g_stats_mu);
    g_stats.scan_iterations += iter;
    g_stats.kd_searches += (long long)iter * N;
    g_stats.kd_leaves += leaves;
    g_stats.kd_splits += splits;
    pthread_mutex_unlock(&g_stats_mu);
    free(rows);
    free(cnts[0]);
    free(cnts[1]);
    return iter;
}

int ora_scan_reduce(int N, int D, const float *X, int K, float *C, int *clusters, int precision) {
    return ora_scan_reduce_n(N, D, X, K, C, clusters, precision, 100);
}

/* ---- KNNFit core (encoder.lpr:945-965) --------------------------------- */
void ora_knnfit_assign(int R4, int CS, const float *cand, int N, const float *q, float eps, int *best) {
    float **rows = (float **)malloc(sizeof(float *) * (size_t)R4);
    for (int j = 0; j < R4; j++) rows[j] = (float *)cand + (size_t)j * CS;
    ora_kdtree *kdt = ora_kdtree_create(rows, R4, CS, 1);
    int idxs[64];
    float errs[64];
    for (int i = 0; i < N; i++) {
        ora_kdtree_pri_search_multi(kdt, idxs, errs, 64, q + (size_t)i * CS, 0.0f);
        int b = idxs[0];
        float s0 = sqrtf(errs[0] / (float)CS);
        for (int j = 0; j < 64; j++) {
            if (idxs[j] >= 0 && idxs[j] <= b - 1) {
                float sj = sqrtf(errs[j] / (float)CS);
                float d = s0 > sj ? s0 - sj : sj - s0;
                if (d <= eps) b = idxs[j];
            }
        }
        best[i] = b;
    }
    ora_kdtree_destroy(kdt);
    free(rows);
}

/* ---- encoder state ------------------------------------------------------ */
typedef struct {
    gsc_params p;
    int channels, sample_rate, sample_count;
    double **filtered; /* [ch][sample] */
    int frame_count;
    int *fr_start, *fr_end;
    int block;
} enc_t;

typedef struct {
    /* per chunk (chunkRefs order = i*C + ch) */
    int n;
    double *src;   /* n*CS */
    double *dct;   /* n*2CS */
    int16_t *dst;  /* n*CS */
    int *atten, *neg, *rev, *red;
    /* reduced chunks */
    int r;
    double *rsrc;
    int16_t *rdst;
    int *ratten, *rneg, *rrev, *ruse, *rindex;
    int atten_div;
    int scan_iters;
} frame_t;

static void frame_free(frame_t *f) {
    free(f->src); free(f->dct); free(f->dst); free(f->atten); free(f->neg); free(f->rev); free(f->red);
    free(f->rsrc); free(f->rdst); free(f->ratten); free(f->rneg); free(f->rrev); free(f->ruse); free(f->rindex);
    memset(f, 0, sizeof(*f));
}

/* Pascal integer div (truncates toward zero) */
static int pdiv(int a, int b) { return a / b; }

/* TEncoder.Load (encoder.lpr:1111-1152) + PrepareFrames (encoder.lpr:1294-1429) */
static int enc_prepare(enc_t *e, const uint8_t *wav, size_t len) {
    if (len < 44) return -1;
    e->sample_rate = (int)(wav[0x18] | (wav[0x19] << 8) | (wav[0x1a] << 16) | ((uint32_t)wav[0x1b] << 24));
    e->channels = wav[0x16] | (wav[0x17] << 8);
    if (e->channels <= 0) return -1;
    const gsc_params *p = &e->p;
    if (p->chunk_blend != 0 || p->python_reduce) return -2; /* out of scope */
    int sc = (int)((len - 44) / (2 * (size_t)e->channels));
    /* MakeBandGlobalData (encoder.lpr:1241-1273), CBandCount = 1 */
    double hc = p->high_cut < (double)e->sample_rate / 2 ? p->high_cut : (double)e->sample_rate / 2;
    double fcl = p->low_cut / (double)e->sample_rate;
    double fch = hc / (double)e->sample_rate;
    if (fcl > 0.0 || fch < 0.5) return -3; /* band-pass filter active: out of scope */
    long long us = fpc_round(0.25 / fch);
    int under = us > 1 ? (int)us : 1;
    if (under != 1) return -3;
    e->block = under * (p->chunk_size - p->chunk_blend);
    int psc = sc;
    int padded = (pdiv(sc - 1, e->block) + 1) * e->block; /* Pascal div (encoder.lpr:1319) */
    e->sample_count = padded;
    e->filtered = (double **)malloc(sizeof(double *) * (size_t)e->channels);
    const uint8_t *d = wav + 44;
    for (int c = 0; c < e->channels; c++) {
        e->filtered[c] = (double *)calloc((size_t)(padded > 0 ? padded : 1), sizeof(double));
        for (int i = 0; i < psc; i++) {
            const uint8_t *b = d + ((size_t)i * e->channels + c) * 2;
            int16_t s = (int16_t)(b[0] | (b[1] << 8));
            e->filtered[c][i] = (double)s / 32767.0;
        }
    }
    int SC = e->sample_count, CH = e->channels;
    int frame_count = (int)fpc_ceil((double)SC / ((double)e->sample_rate * (p->frame_length / 1000.0)));
    /* ChunksPerFrame loop (encoder.lpr:1337-1351) */
    int cpf = p->chunks_per_frame;
    long long projected = 2147483647LL;
    if (p->bit_rate > 0)
        projected = (long long)ceil(((double)SC / (double)e->sample_rate) * ((double)p->bit_rate * 1024.0 / 8.0));
    cpf++;
    for (;;) {
        cpf--;
        double band_cost = ((double)SC * (double)CH * (log2((double)cpf) + (1 + 2) + 1 + 1)) /
                           (8.0 * (double)(p->chunk_size - p->chunk_blend) * (double)under);
        double frame_cost = (double)(cpf * p->chunk_size) * (double)p->chunk_bit_depth / 8.0 + (double)cpf * 4.0 / 8.0 +
                            (4 * 2 + 4 + 1 * 4);
        long long tent = fpc_round(0.0 + band_cost * 0.8 + (double)frame_count * frame_cost);
        int tent32 = (int)(int32_t)tent;
        if ((long long)tent32 <= projected || cpf <= 1) break;
    }
    e->p.chunks_per_frame = cpf;
    /* pass 2: RMS-power balanced frame cuts */
    double avg = 0.0;
    for (int j = 0; j < CH; j++)
        for (int i = 0; i < SC; i++) {
            double v = e->filtered[j][i]; /* makeFloatSample(srcData) == filtered when unfiltered */
            avg += v * v;
        }
    avg = sqrt(avg / (double)(SC * CH));
    double total = 0.0;
    for (int i = 0; i < SC; i++) {
        double smp = 0.0;
        for (int j = 0; j < CH; j++) smp += e->filtered[j][i] * e->filtered[j][i];
        smp = sqrt(smp / (double)CH);
        total += 1.0 - (avg + (smp - avg) * p->vfr);
    }
    double per_frame = total / (double)frame_count;
    int cap = 16;
    e->fr_start = (int *)malloc(sizeof(int) * (size_t)cap);
    e->fr_end = (int *)malloc(sizeof(int) * (size_t)cap);
    int k = 0, next = 0;
    double cur = 0.0;
    for (int i = 0; i < SC; i++) {
        double smp = 0.0;
        for (int j = 0; j < CH; j++) smp += e->filtered[j][i] * e->filtered[j][i];
        smp = sqrt(smp / (double)CH);
        cur += 1.0 - (avg + (smp - avg) * p->vfr);
        if ((i % e->block == 0) && (cur >= per_frame)) {
            if (k + 1 >= cap) {
                cap *= 2;
                e->fr_start = (int *)realloc(e->fr_start, sizeof(int) * (size_t)cap);
                e->fr_end = (int *)realloc(e->fr_end, sizeof(int) * (size_t)cap);
            }
            e->fr_start[k] = next;
            e->fr_end[k] = i - 1;
            cur = 0.0;
            next = i;
            k++;
        }
    }
    if (k + 1 >= cap) {
        cap *= 2;
        e->fr_start = (int *)realloc(e->fr_start, sizeof(int) * (size_t)cap);
        e->fr_end = (int *)realloc(e->fr_end, sizeof(int) * (size_t)cap);
    }
    e->fr_start[k] = next;
    e->fr_end[k] = SC - 1;
    k++;
    e->frame_count = k;
    return 0;
}

static void enc_free(enc_t *e) {
    if (e->filtered) {
        for (int c = 0; c < e->channels; c++) free(e->filtered[c]);
        free(e->filtered);
    }
    free(e->fr_start);
    free(e->fr_end);
}

/* TFrame.MakeChunks / TBand.MakeChunks (encoder.lpr:467-485,607-619) */
static void frame_make_chunks(const enc_t *e, frame_t *f, int start, int sc) {
    int CS = e->p.chunk_size, CH = e->channels;
    int chunk_count = pdiv(sc - 1, CS) + 1;
    int n = chunk_count * CH;
    f->n = n;
    f->src = (double *)calloc((size_t)n * CS, sizeof(double));
    f->dct = (double *)calloc((size_t)n * 2 * CS, sizeof(double));
    f->dst = (int16_t *)calloc((size_t)n * CS, sizeof(int16_t));
    f->atten = (int *)calloc((size_t)n, sizeof(int));
    f->neg = (int *)calloc((size_t)n, sizeof(int));
    f->rev = (int *)calloc((size_t)n, sizeof(int));
    f->red = (int *)calloc((size_t)n, sizeof(int));
    double law = 1.0 / (double)f->atten_div;
    for (int i = 0; i < chunk_count; i++)
        for (int j = 0; j < CH; j++) {
            int c = i * CH + j;
            double *s = f->src + (size_t)c * CS;
            for (int k = 0; k < CS; k++) {
                int pos = i * CS + k;
                s[k] = (pos >= sc) ? 0.0 : 0.0 + e->filtered[j][start + pos];
            }
            dst_attributes(CS, s, law, &f->atten[c], &f->neg[c], &f->rev[c]);
            for (int k = 0; k < CS; k++)
                f->dst[(size_t)c * CS + k] =
                    ora_make_output_sample(s[k], e->p.chunk_bit_depth, f->atten[c], f->neg[c], law);
            ora_chunk_features(CS, s, f->neg[c], f->rev[c], f->dct + (size_t)c * 2 * CS);
        }
}

typedef struct {
    float *dataset, *yakmo, *scan;
    int *clusters;
} reduce_trace;

/* TFrame.Reduce (encoder.lpr:785-913) */
static void frame_reduce(const enc_t *e, frame_t *f, reduce_trace *tr) {
    int CS = e->p.chunk_size, D = 2 * CS, K = e->p.chunks_per_frame, N = f->n;
    int bd = e->p.chunk_bit_depth;
    double law = 1.0 / (double)f->atten_div;
    float *X = (float *)malloc(sizeof(float) * (size_t)N * D);
    for (size_t i = 0; i < (size_t)N * D; i++) X[i] = (float)f->dct[i];
    if (tr && tr->dataset) memcpy(tr->dataset, X, sizeof(float) * (size_t)N * D);
    if (e->p.precision > 0 && N > K) {
        float *C = (float *)malloc(sizeof(float) * (size_t)K * D);
        int *clusters = (int *)malloc(sizeof(int) * (size_t)N);
        ora_yakmo_seed_means(N, D, X, K, C, clusters);
        if (tr && tr->yakmo) memcpy(tr->yakmo, C, sizeof(float) * (size_t)K * D);
        f->scan_iters = ora_scan_reduce(N, D, X, K, C, clusters, e->p.precision);
        if (tr && tr->scan) memcpy(tr->scan, C, sizeof(float) * (size_t)K * D);
        if (tr && tr->clusters) memcpy(tr->clusters, clusters, sizeof(int) * (size_t)N);
        /* cluster means of canonicalised srcData (encoder.lpr:845-864) */
        double *acc = (double *)calloc((size_t)K * CS, sizeof(double));
        int *count = (int *)calloc((size_t)K, sizeof(int));
        for (int j = 0; j < N; j++) {
            int c = clusters[j];
            const double *s = f->src + (size_t)j * CS;
            for (int k = 0; k < CS; k++)
                acc[(size_t)c * CS + k] += s[f->rev[j] ? CS - 1 - k : k] * (f->neg[j] ? -1.0 : 1.0);
            count[c]++;
        }
        for (int i = 0; i < K; i++)
            for (int k = 0; k < CS; k++) {
                double y = (double)count[i];
                double v = fpc_iszero(y) ? 0.0 : acc[(size_t)i * CS + k] / y;
                C[(size_t)i * D + k] = (float)v;
            }
        int *perm = (int *)malloc(sizeof(int) * (size_t)K);
        ora_sort_count_desc(K, count, perm);
        f->r = K;
        f->rsrc = (double *)calloc((size_t)K * CS, sizeof(double));
        f->rdst = (int16_t *)calloc((size_t)K * CS, sizeof(int16_t));
        f->ratten = (int *)calloc((size_t)K, sizeof(int));
        f->rneg = (int *)calloc((size_t)K, sizeof(int));
        f->rrev = (int *)calloc((size_t)K, sizeof(int));
        for (int i = 0; i < K; i++) {
            double *rs = f->rsrc + (size_t)i * CS;
            for (int j = 0; j < CS; j++) {
                double v = (double)C[(size_t)perm[i] * D + j];
                rs[j] = isnan(v) ? 0.0 : v;
            }
            dst_attributes(CS, rs, law, &f->ratten[i], &f->rneg[i], &f->rrev[i]);
            for (int j = 0; j < CS; j++)
                f->rdst[(size_t)i * CS + j] = ora_make_output_sample(rs[j], bd, f->ratten[i], f->rneg[i], law);
        }
        free(perm);
        free(acc);
        free(count);
        free(C);
        free(clusters);
    } else {
        f->r = N;
        f->rsrc = (double *)calloc((size_t)N * CS, sizeof(double));
        f->rdst = (int16_t *)calloc((size_t)N * CS, sizeof(int16_t));
        f->ratten = (int *)calloc((size_t)N, sizeof(int));
        f->rneg = (int *)calloc((size_t)N, sizeof(int));
        f->rrev = (int *)calloc((size_t)N, sizeof(int));
        for (int i = 0; i < N; i++) {
            double *rs = f->rsrc + (size_t)i * CS;
            memcpy(rs, f->src + (size_t)i * CS, sizeof(double) * (size_t)CS);
            dst_attributes(CS, rs, law, &f->ratten[i], &f->rneg[i], &f->rrev[i]);
            for (int j = 0; j < CS; j++)
                f->rdst[(size_t)i * CS + j] = ora_make_output_sample(rs[j], bd, f->ratten[i], f->rneg[i], law);
        }
    }
    f->ruse = (int *)calloc((size_t)f->r, sizeof(int));
    f->rindex = (int *)calloc((size_t)f->r, sizeof(int));
    free(X);
}

typedef struct {
    float *cand, *query;
    int *best;
    float eps;
} knn_trace;

/* TFrame.KNNFit (encoder.lpr:915-978); leaves f->red[] = final position */
static void frame_knnfit(const enc_t *e, frame_t *f, knn_trace *tr) {
    int CS = e->p.chunk_size, bd = e->p.chunk_bit_depth, R = f->r, N = f->n;
    double law = 1.0 / (double)f->atten_div;
    float *cand = (float *)malloc(sizeof(float) * (size_t)4 * R * CS);
    for (int i = 0; i < 2 * R; i++)
        for (int j = 0; j < CS; j++) {
            int c = i >> 1;
            cand[(size_t)(i * 2 + 0) * CS + j] =
                (float)ora_make_float_sample(f->rdst[(size_t)c * CS + j], bd, f->ratten[c], i & 1, law);
            cand[(size_t)(i * 2 + 1) * CS + j] =
                (float)ora_make_float_sample(f->rdst[(size_t)c * CS + CS - 1 - j], bd, f->ratten[c], i & 1, law);
        }
    float acc = 1.0f;
    for (int j = 0; j <= C_MAX_ATTENUATION; j++) acc = (float)((double)acc + (double)j * law);
    float e1 = 1.0f / ((float)(1 << bd) * acc);
    float e2 = (float)(1.0 / 32767.0);
    float eps = e1 > e2 ? e1 : e2;
    float *q = (float *)malloc(sizeof(float) * (size_t)N * CS);
    for (size_t i = 0; i < (size_t)N * CS; i++) q[i] = (float)f->src[i];
    int *best = (int *)malloc(sizeof(int) * (size_t)N);
    ora_knnfit_assign(4 * R, CS, cand, N, q, eps, best);
    if (tr) {
        if (tr->cand) memcpy(tr->cand, cand, sizeof(float) * (size_t)4 * R * CS);
        if (tr->query) memcpy(tr->query, q, sizeof(float) * (size_t)N * CS);
        if (tr->best) memcpy(tr->best, best, sizeof(int) * (size_t)N);
        tr->eps = eps;
    }
    for (int i = 0; i < N; i++) {
        int b = best[i];
        f->neg[i] = (b & 2) != 0;
        f->rev[i] = (b & 1) != 0;
        f->red[i] = b >> 2;
        f->ruse[b >> 2]++;
    }
    /* delete unused, sort by useCount desc (FPC QuickSort), reindex */
    int *alive = (int *)malloc(sizeof(int) * (size_t)R);
    int na = 0;
    for (int i = 0; i < R; i++)
        if (f->ruse[i] != 0) alive[na++] = i;
    int *cnt = (int *)malloc(sizeof(int) * (size_t)(na > 0 ? na : 1));
    for (int i = 0; i < na; i++) cnt[i] = f->ruse[alive[i]];
    int *perm = (int *)malloc(sizeof(int) * (size_t)(na > 0 ? na : 1));
    ora_sort_count_desc(na, cnt, perm);
    for (int i = 0; i < R; i++) f->rindex[i] = -1;
    for (int i = 0; i < na; i++) f->rindex[alive[perm[i]]] = i;
    /* compact the reduced list into final order */
    double *nsrc = (double *)calloc((size_t)(na > 0 ? na : 1) * CS, sizeof(double));
    int16_t *ndst = (int16_t *)calloc((size_t)(na > 0 ? na : 1) * CS, sizeof(int16_t));
    int *natt = (int *)calloc((size_t)(na > 0 ? na : 1), sizeof(int));
    for (int i = 0; i < na; i++) {
        int o = alive[perm[i]];
        memcpy(nsrc + (size_t)i * CS, f->rsrc + (size_t)o * CS, sizeof(double) * (size_t)CS);
        memcpy(ndst + (size_t)i * CS, f->rdst + (size_t)o * CS, sizeof(int16_t) * (size_t)CS);
        natt[i] = f->ratten[o];
    }
    for (int i = 0; i < N; i++) f->red[i] = f->rindex[f->red[i]];
    free(f->rsrc);
    free(f->rdst);
    free(f->ratten);
    f->rsrc = nsrc;
    f->rdst = ndst;
    f->ratten = natt;
    f->r = na;
    free(alive);
    free(cnt);
    free(perm);
    free(cand);
    free(q);
    free(best);
}

/* ---- byte buffer -------------------------------------------------------- */
typedef struct {
    uint8_t *b;
    size_t n, cap;
} buf_t;
static void put(buf_t *o, const void *p, size_t n) {
    if (o->n + n > o->cap) {
        o->cap = (o->n + n) * 2 + 64;
        o->b = (uint8_t *)realloc(o->b, o->cap);
    }
    memcpy(o->b + o->n, p, n);
    o->n += n;
}
static void put8(buf_t *o, unsigned v) { uint8_t x = (uint8_t)v; put(o, &x, 1); }
static void put16(buf_t *o, unsigned v) { uint8_t x[2] = {(uint8_t)v, (uint8_t)(v >> 8)}; put(o, x, 2); }
static void put32(buf_t *o, uint32_t v) {
    uint8_t x[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)};
    put(o, x, 4);
}
static int bsr_word(unsigned v) {
    int r = 0;
    while (v >>= 1) r++;
    return r;
}

/* TFrame.SaveStream (encoder.lpr:980-1107) */
static void frame_save(const enc_t *e, const frame_t *f, buf_t *o) {
    int CS = e->p.chunk_size, bd = e->p.chunk_bit_depth, CH = e->channels;
    put16(o, (unsigned)((CH << 8) | 1));
    put16(o, (unsigned)(f->r | (0 << 13)));
    put16(o, (unsigned)((CS << 8) | bd));
    put32(o, (uint32_t)((e->p.chunk_blend << 24) | e->sample_rate));
    put16(o, (unsigned)f->atten_div);
    int R = f->r;
    for (int j = 0; j < R / 2; j++) put8(o, (unsigned)((f->ratten[2 * j] << 4) | f->ratten[2 * j + 1]));
    if (R & 1) put8(o, (unsigned)(f->ratten[R - 1] << 4));
    if (bd == 8) {
        for (int j = 0; j < R; j++)
            for (int k = 0; k < CS; k++) put8(o, (unsigned)((f->rdst[(size_t)j * CS + k] + 128) & 0xff));
    } else {
        for (int j = 0; j < R; j++) {
            const int16_t *d = f->rdst + (size_t)j * CS;
            for (int k = 0; k < CS / 2; k++) {
                int s1 = d[2 * k] + 2048, s2 = d[2 * k + 1] + 2048;
                put8(o, (unsigned)(((s1 >> 4) & 0xf0) | ((s2 >> 8) & 0x0f)));
                put8(o, (unsigned)(s1 & 0xff));
                put8(o, (unsigned)(s2 & 0xff));
            }
            if (CS & 1) {
                int s1 = d[CS - 1] + 2048;
                put8(o, (unsigned)((s1 >> 4) & 0xf0));
                put8(o, (unsigned)(s1 & 0xff));
            }
        }
    }
    put32(o, (uint32_t)(f->n / CH));
    int bit_cnt = 0;
    uint32_t bits = 0;
    for (int j = 0; j < f->n; j++) {
        int idx = f->red[j];
        int vc = idx == 0 ? 0 : bsr_word((unsigned)idx) / 3;
        int pvc = -1;
        if (j >= 1) {
            int pidx = f->red[j - 1];
            pvc = pidx == 0 ? 0 : bsr_word((unsigned)pidx) / 3;
        }
        uint64_t code = 0;
        int cs_ = 0;
        code |= (uint64_t)(f->neg[j] ? 1 : 0) << cs_;
        cs_ += 1;
        code |= (uint64_t)(f->rev[j] ? 1 : 0) << cs_;
        cs_ += 1;
        if (vc == pvc) {
            cs_ += 1;
        } else {
            code |= (uint64_t)1 << cs_;
            cs_ += 1;
            code |= (uint64_t)vc << cs_;
            cs_ += 2;
        }
        for (int k = vc; k >= 0; k--) {
            code |= (uint64_t)((idx >> (k * 3)) & 7) << cs_;
            cs_ += 3;
        }
        bits = (uint32_t)(bits | ((uint32_t)code << bit_cnt));
        bit_cnt += cs_;
        if (bit_cnt >= 16) {
            bit_cnt -= 16;
            put16(o, bits & 0xffff);
            bits >>= 16;
        }
    }
    if (bit_cnt > 0) put16(o, bits & 0xffff);
}

/* make16BitSample (encoder.lpr:1638-1641): EnsureRange(round(smp * High(SmallInt))) */
static int16_t make16(double smp) {
    return (int16_t)clampll(fpc_round(smp * 32767.0), -32768, 32767);
}

/* Reconstruction of one frame (f4): TBand.MakeDstData (encoder.lpr:487-522;
 * CBandCount = 1, underSample = 1, ChunkBlend = 0) writes each final chunk's
 * CS samples, makeFloatSample of its reduced chunk (reversed / negated as
 * KNNFit chose), at the channel's running position, dropping positions past
 * the frame; TEncoder.MakeDstData (encoder.lpr:1518-1582) sums the (single)
 * band into floatDst and stores make16BitSample.  recon is interleaved
 * [sample][channel] over the padded SampleCount, as SaveWAV writes it
 * (encoder.lpr:1154-1179). */
static void frame_recon(const enc_t *e, const frame_t *f, int start, int sc, int16_t *recon) {
    int CS = e->p.chunk_size, CH = e->channels, bd = e->p.chunk_bit_depth;
    double law = 1.0 / (double)f->atten_div;
    for (int i = 0; i < f->n; i++) {
        int ch = i % CH, chunk = i / CH, c = f->red[i];
        for (int j = 0; j < CS; j++) {
            int pos = chunk * CS + j;
            int16_t v = f->rdst[(size_t)c * CS + (f->rev[i] ? CS - 1 - j : j)];
            double smp = ora_make_float_sample(v, bd, f->ratten[c], f->neg[i], law);
            if (pos < sc) recon[(size_t)(start + pos) * CH + ch] = make16(0.0 + (0.0 + smp));
        }
    }
}

/* DoFrame (encoder.lpr:1433-1447) */
static void do_frame_r(const enc_t *e, int fi, buf_t *o, frame_t *keep, reduce_trace *rtr, knn_trace *ktr,
                       int16_t *recon);
static void do_frame(const enc_t *e, int fi, buf_t *o, frame_t *keep, reduce_trace *rtr, knn_trace *ktr) {
    do_frame_r(e, fi, o, keep, rtr, ktr, NULL);
}
static void do_frame_r(const enc_t *e, int fi, buf_t *o, frame_t *keep, reduce_trace *rtr, knn_trace *ktr,
                       int16_t *recon) {
    frame_t f;
    memset(&f, 0, sizeof(f));
    int start = e->fr_start[fi], end = e->fr_end[fi];
    int sc = end - start + 1;
    /* FindAttenuationDivider operates on channel rows from `start` */
    {
        int CH = e->channels;
        double *tmp = (double *)malloc(sizeof(double) * (size_t)CH * (size_t)(sc > 0 ? sc : 1));
        for (int c = 0; c < CH; c++)
            for (int i = 0; i < sc; i++) tmp[(size_t)c * sc + i] = e->filtered[c][start + i];
        f.atten_div = ora_find_atten_divider(tmp, CH, sc, sc, e->p.chunk_size, e->p.chunk_bit_depth);
        free(tmp);
    }
    frame_make_chunks(e, &f, start, sc);
    frame_reduce(e, &f, rtr);
    frame_knnfit(e, &f, ktr);
    if (o) frame_save(e, &f, o);
    if (recon) frame_recon(e, &f, start, sc, recon);
    if (keep) *keep = f;
    else frame_free(&f);
}

typedef struct {
    const enc_t *e;
    buf_t *outs;
    int16_t *recon; /* optional: interleaved reconstruction */
    int next, end;
    pthread_mutex_t mu;
} pool_t;

static void *worker(void *arg) {
    pool_t *pl = (pool_t *)arg;
    for (;;) {
        pthread_mutex_lock(&pl->mu);
        int fi = pl->next++;
        pthread_mutex_unlock(&pl->mu);
        if (fi >= pl->end) break;
        do_frame_r(pl->e, fi, &pl->outs[fi], NULL, NULL, NULL, pl->recon);
    }
    return NULL;
}

/* Frames [frame_begin, frame_end) of the whole-file encode (frame_end < 0 =>
 * all); their TFrame.SaveStream bytes concatenated in frame order
 * (encoder.lpr:1181-1215 writes frames in order).  Used by the multi-rank
 * sharding tests: the concatenation over ranks equals ora_encode. */
static int encode_frames_r(const uint8_t *wav, size_t wav_len, const gsc_params *p, int frame_begin, int frame_end,
                           int threads, uint8_t **out, size_t *out_len, int *frame_count, int16_t **recon,
                           size_t *recon_len, double *psy);
int ora_encode_frames(const uint8_t *wav, size_t wav_len, const gsc_params *p, int frame_begin, int frame_end,
                      int threads, uint8_t **out, size_t *out_len, int *frame_count) {
    return encode_frames_r(wav, wav_len, p, frame_begin, frame_end, threads, out, out_len, frame_count, NULL, NULL,
                           NULL);
}

/* ComputePsyADelta (encoder.lpr:1862-1880) -> CompareEuclidean on Double
 * arrays (encoder.lpr:1803-1814): sqrt(sum((src - dst)^2) / len), the sum
 * sequential in channel-major order over the padded SampleCount. */
static double psy_a_delta(const uint8_t *wav, size_t wav_len, int CH, int SC, const int16_t *recon) {
    int psc = (int)((wav_len - 44) / (2 * (size_t)CH));
    double acc = 0.0;
    for (int j = 0; j < CH; j++)
        for (int i = 0; i < SC; i++) {
            int16_t s = 0;
            if (i < psc) {
                const uint8_t *b = wav + 44 + ((size_t)i * CH + j) * 2;
                s = (int16_t)(b[0] | (b[1] << 8));
            }
            double d = (double)s - (double)recon[(size_t)i * CH + j];
            acc += d * d;
        }
    return sqrt(acc / (double)((long long)CH * SC));
}

int ora_encode_recon(const uint8_t *wav, size_t wav_len, const gsc_params *p, int threads, uint8_t **out,
                     size_t *out_len, int16_t **recon, size_t *recon_len, double *psy) {
    return encode_frames_r(wav, wav_len, p, 0, -1, threads, out, out_len, NULL, recon, recon_len, psy);
}

static int encode_frames_r(const uint8_t *wav, size_t wav_len, const gsc_params *p, int frame_begin, int frame_end,
                           int threads, uint8_t **out, size_t *out_len, int *frame_count, int16_t **recon,
                           size_t *recon_len, double *psy) {
    enc_t e;
    memset(&e, 0, sizeof(e));
    e.p = *p;
    int rc = enc_prepare(&e, wav, wav_len);
    if (rc != 0) {
        enc_free(&e);
        return rc;
    }
    if (frame_count) *frame_count = e.frame_count;
    if (frame_begin < 0) frame_begin = 0;
    if (frame_end < 0 || frame_end > e.frame_count) frame_end = e.frame_count;
    (void)get_trig(e.p.chunk_size);
    pthread_mutex_lock(&g_stats_mu);
    memset(&g_stats, 0, sizeof(g_stats));
    g_stats.frame_count = e.frame_count;
    pthread_mutex_unlock(&g_stats_mu);
    buf_t *outs = (buf_t *)calloc((size_t)(e.frame_count > 0 ? e.frame_count : 1), sizeof(buf_t));
    int nf = frame_end - frame_begin;
    if (threads <= 0) threads = 1;
    if (threads > nf) threads = nf;
    pool_t pl;
    pl.e = &e;
    pl.outs = outs;
    pl.recon = recon ? (int16_t *)calloc((size_t)e.sample_count * (size_t)e.channels + 1, sizeof(int16_t)) : NULL;
    pl.next = frame_begin;
    pl.end = frame_end;
    pthread_mutex_init(&pl.mu, NULL);
    if (threads <= 1) {
        worker(&pl);
    } else {
        pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
        for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, worker, &pl);
        for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
        free(th);
    }
    pthread_mutex_destroy(&pl.mu);
    buf_t all = {0};
    for (int i = frame_begin; i < frame_end; i++) {
        put(&all, outs[i].b, outs[i].n);
        free(outs[i].b);
    }
    free(outs);
    if (recon) {
        *recon = pl.recon;
        *recon_len = (size_t)e.sample_count * (size_t)e.channels;
        if (psy) *psy = psy_a_delta(wav, wav_len, e.channels, e.sample_count, pl.recon);
    }
    enc_free(&e);
    if (!all.b) all.b = (uint8_t *)malloc(1);
    *out = all.b;
    *out_len = all.n;
    return 0;
}

int ora_encode(const uint8_t *wav, size_t wav_len, const gsc_params *p, int threads, uint8_t **out, size_t *out_len) {
    return ora_encode_frames(wav, wav_len, p, 0, -1, threads, out, out_len, NULL);
}

int ora_trace_frame(const uint8_t *wav, size_t wav_len, const gsc_params *p, int frame_idx, ora_frame_trace *tr) {
    enc_t e;
    memset(&e, 0, sizeof(e));
    e.p = *p;
    int rc = enc_prepare(&e, wav, wav_len);
    if (rc != 0) {
        enc_free(&e);
        return rc;
    }
    if (frame_idx < 0 || frame_idx >= e.frame_count) {
        enc_free(&e);
        return -4;
    }
    int start = e.fr_start[frame_idx], end = e.fr_end[frame_idx];
    int sc = end - start + 1;
    int CS = e.p.chunk_size, CH = e.channels, K = e.p.chunks_per_frame;
    int N = (pdiv(sc - 1, CS) + 1) * CH;
    memset(tr, 0, sizeof(*tr));
    tr->N = N;
    tr->K = K;
    tr->D = 2 * CS;
    tr->CS = CS;
    reduce_trace rt;
    rt.dataset = (float *)malloc(sizeof(float) * (size_t)N * 2 * CS);
    rt.yakmo = (float *)calloc((size_t)K * 2 * CS, sizeof(float));
    rt.scan = (float *)calloc((size_t)K * 2 * CS, sizeof(float));
    rt.clusters = (int *)calloc((size_t)N, sizeof(int));
    int R = N > K ? K : N;
    knn_trace kt;
    kt.cand = (float *)malloc(sizeof(float) * (size_t)4 * R * CS);
    kt.query = (float *)malloc(sizeof(float) * (size_t)N * CS);
    kt.best = (int *)malloc(sizeof(int) * (size_t)N);
    frame_t f;
    do_frame(&e, frame_idx, NULL, &f, &rt, &kt);
    tr->atten_div = f.atten_div;
    tr->scan_iters = f.scan_iters;
    tr->reduced_count = R;
    tr->dataset = rt.dataset;
    tr->yakmo_centroids = rt.yakmo;
    tr->scan_centroids = rt.scan;
    tr->clusters = rt.clusters;
    tr->knn_best = kt.best;
    tr->knn_cand = kt.cand;
    tr->knn_query = kt.query;
    tr->knn_eps = kt.eps;
    frame_free(&f);
    enc_free(&e);
    return 0;
}

/* ---- decoder restatement (decoder/decoder.lpr:37-220) ------------------- */
long ora_decode(const uint8_t *g, size_t len, int16_t **pcm, int *channels, int *rate) {
    size_t pos = 0;
    buf_t o = {0};
    const double attr_mul = (double)fpc_round(32768.0 * (32767.0 / 2047.0));
    int ch = 0, sr = 0;
    while (pos < len) {
        if (pos + 12 > len) break;
        int ver = g[pos];
        ch = g[pos + 1];
        int count = (g[pos + 2] | (g[pos + 3] << 8)) & 0x1fff;
        int bd = g[pos + 4], cs = g[pos + 5];
        uint32_t srw = (uint32_t)(g[pos + 6] | (g[pos + 7] << 8) | (g[pos + 8] << 16) | ((uint32_t)g[pos + 9] << 24));
        sr = (int)(srw & 0xffffff);
        int adiv = g[pos + 10] | (g[pos + 11] << 8);
        pos += 12;
        double law = 1.0 / (double)adiv, lacc = 1.0;
        int lut[2][16];
        for (int i = 0; i <= 15; i++) {
            lacc += law * (double)i;
            lut[0][i] = (int)fpc_round(attr_mul / lacc);
            lut[1][i] = -(int)fpc_round(attr_mul / lacc);
        }
        int *att = (int *)calloc((size_t)(count > 0 ? count : 1), sizeof(int));
        int16_t *chunks = (int16_t *)calloc((size_t)(count > 0 ? count : 1) * (size_t)(cs > 0 ? cs : 1), 2);
        for (int i = 0; i < count / 2; i++) {
            int b = g[pos++];
            att[2 * i] = (b & 0xf0) >> 4;
            att[2 * i + 1] = b & 0x0f;
        }
        if (count & 1) att[count - 1] = (g[pos++] & 0xf0) >> 4;
        if (bd == 8) {
            for (int i = 0; i < count; i++)
                for (int j = 0; j < cs; j++) {
                    int b = g[pos++];
                    chunks[i * cs + j] = (int16_t)((b - 128) * 2047 / 127);
                }
        } else {
            for (int i = 0; i < count; i++) {
                for (int j = 0; j < cs / 2; j++) {
                    int b = g[pos++];
                    int s1 = g[pos++] | ((b & 0xf0) << 4);
                    int s2 = g[pos++] | ((b & 0x0f) << 8);
                    chunks[i * cs + 2 * j] = (int16_t)(s1 - 2048);
                    chunks[i * cs + 2 * j + 1] = (int16_t)(s2 - 2048);
                }
                if (cs & 1) {
                    int b = g[pos++];
                    int s1 = g[pos++] | ((b & 0xf0) << 4);
                    chunks[i * cs + cs - 1] = (int16_t)(s1 - 2048);
                }
            }
        }
        uint32_t flen = (uint32_t)(g[pos] | (g[pos + 1] << 8) | (g[pos + 2] << 16) | ((uint32_t)g[pos + 3] << 24));
        pos += 4;
        uint32_t bits = 0;
        int bit_count = 0, vch = -1;
        int cidx[256], cneg[256], crev[256];
#define FILL()                                                      \
    if (bit_count < 16 && pos < len) {                              \
        unsigned w = (unsigned)(g[pos] | (g[pos + 1] << 8));        \
        pos += 2;                                                   \
        bits |= (uint32_t)w << bit_count;                           \
        bit_count += 16;                                            \
    }
#define GET(n_) (tmpv = (int)(bits & ((1u << (n_)) - 1)), bits >>= (n_), bit_count -= (n_), tmpv)
        int tmpv;
        for (uint32_t i = 0; i < flen; i++) {
            for (int k = 0; k < ch; k++) {
                FILL();
                cneg[k] = GET(1) != 0;
                if (ver > 0) crev[k] = GET(1) != 0;
                if (GET(1) != 0) vch = GET(2);
                FILL();
                cidx[k] = 0;
                for (int j = 0; j <= vch; j++) cidx[k] = (cidx[k] << 3) | GET(3);
            }
            for (int j = 0; j < cs; j++)
                for (int k = 0; k < ch; k++) {
                    int a = lut[cneg[k]][att[cidx[k]]];
                    int s = chunks[cidx[k] * cs + (crev[k] ? cs - 1 - j : j)];
                    put16(&o, (unsigned)(((uint32_t)(a * s)) >> 15));
                }
        }
#undef FILL
#undef GET
        if (bit_count >= 16) {
            pos -= 2;
            bit_count -= 16;
        }
        free(att);
        free(chunks);
    }
    *pcm = (int16_t *)o.b;
    if (channels) *channels = ch;
    if (rate) *rate = sr;
    return (long)(o.n / 2);
}
