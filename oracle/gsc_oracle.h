/*
 * ORACLE (test infrastructure only) -- CPU restatement of the SoundChunks
 * encoder (reference encoder/encoder.lpr) from in-memory WAV bytes to .gsc
 * bytes, default path (yakmo + KNNScanReduce + KNNFit, single band).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * call this.  It is the checker the HIP product is compared against and the
 * "port" CPU baseline; it is never part of the product.
 *
 * Pinning status:
 *   - quantisers: pinned by the reference's own KAT test_makeSample
 *     (encoder.lpr:1911-1937), ported in tests/test_oracle_kat.py;
 *   - .gsc layout: pinned by a round trip through a restatement of the
 *     reference decoder (decoder/decoder.lpr:37-220);
 *   - FPC trig/log: constants/tables pinned against the encoder.exe image
 *     (read as data) and mpmath;
 *   - yakmo/ANN: parity unpinned (closed-source DLLs cannot run here).
 */
#ifndef GSC_ORACLE_H
#define GSC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* TEncoder fields set from the command line (encoder.lpr:1486-1509,1985-1998) */
typedef struct {
    int bit_rate;          /* -br, default -1 */
    int precision;         /* -pr, default 3 */
    double low_cut;        /* -lc, default 0 */
    double high_cut;       /* -hc, default 24000 */
    int chunk_bit_depth;   /* -cbd, default 8 */
    int chunk_size;        /* -cs, default 4 */
    int chunks_per_frame;  /* -cpf, default 4096, clamp [256,4096] */
    int reduce_bass_band;  /* !-pbb, default 1 */
    double vfr;            /* -vfr, default 1.0 */
    int chunk_blend;       /* -cb, default 0 */
    double frame_length;   /* -fl, default 4000 ms */
    int python_reduce;     /* -py, unsupported by the oracle */
    int verbose;
} gsc_params;

void ora_default_params(gsc_params *p);
/* argv-style option parsing, same prefix semantics as encoder.lpr:201-227 */
void ora_parse_params(gsc_params *p, int argc, const char *const *argv);

/* Full encode.  Returns 0 on success, -4 when a frame fails SaveStream's
 * Assert(reducedChunks.Count <= 4096) (encoder.lpr:986; -pr0 passthrough
 * frames); *out is malloc'd (free with ora_free).
 * threads <= 0 => 1.  Frames are independent; the result does not depend on
 * the thread count. */
int ora_encode(const uint8_t *wav, size_t wav_len, const gsc_params *p, int threads, uint8_t **out,
               size_t *out_len);
void ora_free(void *p);
/* -py mode: the per-frame labels cluster.py returned (tests/golden/birch_*),
 * labels of frame f at labels + frame_offsets[f]; NULL clears. */
void ora_set_py_labels(const int *labels, const long long *frame_offsets, int nframes);
/* Full encode plus the reconstruction the reference builds after MakeFrames
 * (f4: TBand/TEncoder.MakeDstData, encoder.lpr:487-522,1518-1582) as
 * interleaved 16-bit samples over the padded SampleCount (SaveWAV order), and
 * ComputePsyADelta(srcData, dstData) (encoder.lpr:1862-1880). */
int ora_encode_recon(const uint8_t *wav, size_t wav_len, const gsc_params *p, int threads, uint8_t **out,
                     size_t *out_len, int16_t **recon, size_t *recon_len, double *psy);
/* Frames [frame_begin, frame_end) only (frame_end < 0 => all), concatenated
 * SaveStream bytes; *frame_count (may be NULL) = frames in the file. */
int ora_encode_frames(const uint8_t *wav, size_t wav_len, const gsc_params *p, int frame_begin, int frame_end,
                      int threads, uint8_t **out, size_t *out_len, int *frame_count);
/* The listed frames (distinct indices), concatenated in list order, with each
 * one's byte count in frame_bytes[k]. */
int ora_encode_frame_list(const uint8_t *wav, size_t wav_len, const gsc_params *p, const int *frames, int nframes,
                          int threads, uint8_t **out, size_t *out_len, size_t *frame_bytes, int *frame_count);

/* Statistics of the last ora_encode (process-global, for tests/bench). */
typedef struct {
    int frame_count;
    long long total_chunks;
    long long scan_iterations;   /* sum over frames of KNNScanReduce passes */
    long long kd_searches;       /* KNNScanReduce searches */
    long long kd_leaves;         /* leaves visited by those searches */
    long long kd_splits;         /* split nodes visited by those searches */
} ora_stats;
void ora_get_stats(ora_stats *s);

/* ---- stage entry points (for stage-level parity fixtures) ---------------- */

/* TFrame.FindAttenuationDivider (encoder.lpr:566-605); src[ch*stride + i] */
int ora_find_atten_divider(const double *src, int channels, long stride, int sample_count, int chunk_size,
                           int bit_depth);

/* quantisers (encoder.lpr:1648-1698) */
int16_t ora_make_output_sample(double smp, int bd, int atten, int neg, double law);
double ora_make_float_sample(int16_t smp, int bd, int atten, int neg, double law);
int ora_compute_attenuation(int cs, const double *samples, double law);

/* TChunk feature vector (encoder.lpr:349-363): canonicalise + DCT + cepstrum */
void ora_chunk_features(int cs, const double *src, int neg, int rev, double *dct_out /* 2*cs */);

/* KNNScanReduce (encoder.lpr:699-765) on row-major X[N][D], C[K][D] in/out.
 * Returns the number of passes. */
int ora_scan_reduce(int N, int D, const float *X, int K, float *C, int *clusters, int precision);
/* same, stopping after at most max_passes passes (stage-level tests) */
int ora_scan_reduce_n(int N, int D, const float *X, int K, float *C, int *clusters, int precision, int max_passes);

/* KNNFit core (encoder.lpr:940-965): candidates cand[4R][CS] (already built),
 * queries q[N][CS] f32; writes best candidate index per query. */
void ora_knnfit_assign(int R4, int CS, const float *cand, int N, const float *q, float eps, int *best);

/* FPC TFPSList.QuickSort by count descending: returns the permutation
 * (perm[i] = original position of the item now at i). */
void ora_sort_count_desc(int n, const int *counts, int *perm);

/* Per-frame trace for stage-level golden fixtures: encode only frame
 * `frame_idx` and dump intermediate arrays (any pointer may be NULL).
 * Sizes: dataset N*2CS, yakmo K*2CS, scan K*2CS, clusters N, knn_best N. */
typedef struct {
    int N, K, D, CS, atten_div, scan_iters, reduced_count;
    float *dataset, *yakmo_centroids, *scan_centroids;
    int *clusters;
    int *knn_best; /* 4*reduced_pos + 2*neg + rev, before pruning */
    float *knn_cand;    /* 4R*CS */
    float *knn_query;   /* N*CS */
    float knn_eps;
} ora_frame_trace;
/* Fills the trace (caller frees arrays with ora_free). Returns 0 on success. */
int ora_frame_bounds(const uint8_t *wav, size_t wav_len, const gsc_params *p, int *starts, int *ends, int cap);
int ora_trace_frame(const uint8_t *wav, size_t wav_len, const gsc_params *p, int frame_idx,
                    ora_frame_trace *tr);

/* GSC decoder restatement (decoder.lpr:37-220): .gsc -> interleaved PCM16.
 * Returns number of int16 samples written (malloc'd *pcm), channels/rate out. */
long ora_decode(const uint8_t *gsc, size_t len, int16_t **pcm, int *channels, int *rate);

#ifdef __cplusplus
}
#endif
#endif
