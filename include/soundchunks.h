/*
 * soundchunks_amd -- MI355X-native SoundChunks encode hot path, C ABI.
 *
 * Two layers, both plain C (pointers + sizes, no torch types):
 *
 * 1. The drop-in boundary: exactly the numeric-library surface the reference
 *    binds in encoder/extern.pas:112-123 (yakmo_single.dll + ANN.dll).  On
 *    x86-64 Linux stdcall/cdecl collapse to the SysV ABI.
 *      yakmo_create / yakmo_destroy / yakmo_load_train_data /
 *      yakmo_train_on_data / yakmo_get_centroids    -> extern.pas:112-116
 *      ann_kdtree_create / ann_kdtree_destroy / ann_kdtree_search /
 *      ann_kdtree_pri_search / ann_kdtree_search_multi /
 *      ann_kdtree_pri_search_multi                   -> extern.pas:118-123
 *    Data layout is the reference's: 2-D arrays are float** row-pointer
 *    arrays; ann_kdtree_* keep the caller's row pointers and read the
 *    *current* point values at every search (encoder.lpr:729-745 mutates
 *    centroids between searches of one tree).  All arithmetic runs on the GPU.
 *
 * 2. Frame-level batched entry points (gsc_*): the per-query ANN ABI costs
 *    one host<->device round trip per search, so the encoder itself calls
 *    these, which own the whole Reduce (yakmo + KNNScanReduce) and KNNFit
 *    loops of many frames in one launch each.
 *
 * Errors: functions returning int return 0 on success, <0 on failure;
 * gsc_last_error() describes the last failure of the calling thread.  There is
 * no CPU fallback: without a usable gfx950 device every compute call fails.
 */
#ifndef SOUNDCHUNKS_AMD_H
#define SOUNDCHUNKS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- extern.pas:112-116 (yakmo_single.dll) ----------------------------- */
typedef struct yakmo_t yakmo_t;
/* replaces yakmo_single.dll!yakmo_create @0x180003230 (extern.pas:112) */
yakmo_t *yakmo_create(unsigned int k, unsigned int restartCount, int maxIter, int initType, int initSeed,
                      int doNormalize, int isVerbose);
/* replaces yakmo_destroy @0x180003340 (extern.pas:113) */
void yakmo_destroy(yakmo_t *ay);
/* replaces yakmo_load_train_data @0x180003430 (extern.pas:114); copies rows */
void yakmo_load_train_data(yakmo_t *ay, unsigned int rowCount, unsigned int colCount, float **dataset);
/* replaces yakmo_train_on_data @0x1800034b0 (extern.pas:115); writes labels */
void yakmo_train_on_data(yakmo_t *ay, int *pointToCluster);
/* replaces yakmo_get_centroids @0x180003510 (extern.pas:116) */
void yakmo_get_centroids(yakmo_t *ay, float **centroids);

/* ---- extern.pas:118-123 (ANN.dll) -------------------------------------- */
typedef struct ann_kdtree_t ann_kdtree_t;
/* replaces ANN.dll!ann_kdtree_create @0x180003c50 (extern.pas:118); split 0 = ANN_KD_STD */
ann_kdtree_t *ann_kdtree_create(float **pa, int n, int dd, int bs, int split);
/* replaces ann_kdtree_destroy @0x180003cb0 (extern.pas:119) */
void ann_kdtree_destroy(ann_kdtree_t *akd);
/* replaces ann_kdtree_search @0x180003cd0 (extern.pas:120): k = 1, returns index */
int ann_kdtree_search(ann_kdtree_t *akd, float *q, float eps, float *err);
/* replaces ann_kdtree_pri_search @0x180003d30 (extern.pas:121) */
int ann_kdtree_pri_search(ann_kdtree_t *akd, float *q, float eps, float *err);
/* replaces ann_kdtree_search_multi @0x180003d90 (extern.pas:122) */
void ann_kdtree_search_multi(ann_kdtree_t *akd, int *idxs, float *errs, int cnt, float *q, float eps);
/* replaces ann_kdtree_pri_search_multi @0x180003db0 (extern.pas:123) */
void ann_kdtree_pri_search_multi(ann_kdtree_t *akd, int *idxs, float *errs, int cnt, float *q, float eps);

/* ---- frame-level batched entry points ---------------------------------- */
/* TEncoder options (encoder.lpr:1486-1509, 1985-1998) */
typedef struct {
    int bit_rate;         /* -br, default -1 */
    int precision;        /* -pr, default 3 */
    double low_cut;       /* -lc, default 0 (band-pass filtering unsupported) */
    double high_cut;      /* -hc, default 24000 */
    int chunk_bit_depth;  /* -cbd, default 8 (8 or 12) */
    int chunk_size;       /* -cs, default 4 (1 .. 16) */
    int chunks_per_frame; /* -cpf, default 4096, clamped [256, 4096] */
    int reduce_bass_band; /* !-pbb, default 1 */
    double vfr;           /* -vfr, default 1.0 */
    int chunk_blend;      /* -cb, default 0 (only 0 supported) */
    double frame_length;  /* -fl, default 4000 ms */
    int python_reduce;    /* -py: cluster.py's Birch reducer instead of yakmo + KNNScanReduce */
    int verbose;          /* -v */
} gsc_options;

void gsc_default_options(gsc_options *o);
/* encoder.lpr argv semantics (prefix match, values glued to the flag) */
void gsc_parse_options(gsc_options *o, int argc, const char *const *argv);

/* Whole-file encode: in-memory WAV (44-byte header + PCM16) -> .gsc bytes.
 * *out is allocated by the library; release with gsc_free(). */
int gsc_encode_wav(const uint8_t *wav, size_t wav_len, const gsc_options *o, uint8_t **out, size_t *out_len);

/* Encode plus the reconstruction the reference builds after MakeFrames
 * (encoder.lpr:2019-2031: TEncoder.MakeDstData, ComputePsyADelta, SaveWAV):
 * *recon = the 16-bit signal the .gsc encodes, interleaved [sample][channel]
 * over the padded SampleCount (*recon_len samples; free with gsc_free), as
 * TEncoder.SaveWAV writes it (encoder.lpr:1154-1179); *psy_a_delta =
 * ComputePsyADelta(srcData, dstData) (encoder.lpr:1862-1880).  Reconstruction
 * and the PsyADelta sum run on the device. */
int gsc_encode_wav_recon(const uint8_t *wav, size_t wav_len, const gsc_options *o, uint8_t **out, size_t *out_len,
                         int16_t **recon, size_t *recon_len, double *psy_a_delta);
/* Frame-range encode (multi-GPU sharding): runs the host pre-pass on the
 * whole file, encodes frames [frame_begin, frame_end) only and returns their
 * concatenated TFrame.SaveStream bytes; *frame_count = total frame count. */
int gsc_encode_wav_frames(const uint8_t *wav, size_t wav_len, const gsc_options *o, int frame_begin, int frame_end,
                          uint8_t **out, size_t *out_len, int *frame_count);
int gsc_count_frames(const uint8_t *wav, size_t wav_len, const gsc_options *o, int *frame_count);

/* Prepared WAV: TEncoder.Load + PrepareFrames (encoder.lpr:1111-1152,
 * 1294-1429) run once per job; the frame boundaries of the whole file are then
 * shared by every frame-range encode of that job (one rank per GPU encodes its
 * range without rescanning the file).  gsc_prepare returns NULL on failure
 * (gsc_last_error).  gsc_prepared_frame_chunks writes the chunkRefs count
 * (chunks x channels) of every frame: the weights of the LPT frame sharding. */
typedef struct gsc_prepared gsc_prepared;
gsc_prepared *gsc_prepare(const uint8_t *wav, size_t wav_len, const gsc_options *o);
int gsc_prepared_frame_count(const gsc_prepared *p);
int gsc_prepared_frame_chunks(const gsc_prepared *p, int *chunks);
int gsc_encode_prepared(gsc_prepared *p, int frame_begin, int frame_end, uint8_t **out, size_t *out_len);
/* gsc_encode_prepared, plus each frame's share of the returned bytes.  The
 * range is clamped first (as in gsc_encode_prepared): b = max(frame_begin, 0),
 * e = frame_end < 0 ? frame_count : min(frame_end, frame_count); frame_bytes
 * receives max(e - b, 0) entries, frame_bytes[i - b] for frame i.  A .gsc is
 * the concatenation of its frames' TFrame.SaveStream bytes
 * (encoder.lpr:980-1107, 1181-1215), so the caller can split it per frame
 * (bench.py's per-frame bit-exactness digests).  Every prepared entry point
 * refuses frames outside the range a gsc_prepare_frames handle loaded. */
int gsc_encode_prepared_frames(gsc_prepared *p, int frame_begin, int frame_end, uint8_t **out, size_t *out_len,
                               size_t *frame_bytes);
double gsc_prepared_prepare_ms(const gsc_prepared *p);
/* The frame boundaries PrepareFrames chose: sample index of every frame's
 * first and last sample (gsc_prepared_frame_count entries each). */
int gsc_prepared_frame_bounds(const gsc_prepared *p, int *starts, int *ends);
/* A prepared encoder over boundaries computed elsewhere (one rank runs
 * PrepareFrames on the whole file and broadcasts them): no power scans, and
 * only the samples of frames [frame_begin, frame_end) are loaded, so only
 * that range may be encoded.  frame_end = -1: up to frame_count.  The bounds
 * must be contiguous, block-aligned and cover the file (else NULL). */
gsc_prepared *gsc_prepare_frames(const uint8_t *wav, size_t wav_len, const gsc_options *o, const int *starts,
                                 const int *ends, int frame_count, int frame_begin, int frame_end);
void gsc_prepared_free(gsc_prepared *p);

/* Batch of WAVs as one job (the reference encodes a corpus file by file;
 * encoder.lpr:1431-1451 runs each file's frames on its thread pool): every
 * file gets its own Load + PrepareFrames, then the frames of ALL files form
 * one frame list, so every stage runs one device launch for the whole batch.
 * The files must share channel count, sample rate and the resulting
 * ChunksPerFrame.  A gsc_prepare / gsc_prepare_frames handle is one file
 * (file_count 1).  gsc_prepared_file_frames writes file_count + 1 entries: the
 * first frame of every file, then the total.  gsc_encode_prepared_files
 * encodes frames [frame_begin, frame_end) of the list and also writes, per
 * file, how many of the returned bytes belong to it (files in order; a file's
 * .gsc is its bytes from every range, in range order). */
gsc_prepared *gsc_prepare_many(const uint8_t *const *wavs, const size_t *wav_lens, int file_count,
                               const gsc_options *o);
int gsc_prepared_file_count(const gsc_prepared *p);
int gsc_prepared_file_frames(const gsc_prepared *p, int *first_frame);
int gsc_encode_prepared_files(gsc_prepared *p, int frame_begin, int frame_end, uint8_t **out, size_t *out_len,
                              size_t *file_bytes);

/* Device DSP of one frame (FindAttenuationDivider, encoder.lpr:566-605, and the
 * MakeChunks features, encoder.lpr:467-485): *feat = n_chunks x 2*ChunkSize
 * floats, allocated by the library (gsc_free).  Parity tests. */
int gsc_frame_dsp(const uint8_t *wav, size_t wav_len, const gsc_options *o, int frame, int *atten_div, float **feat,
                  int *n_chunks);

/* Stage entry points on host buffers (row-major), used by parity tests. */
int gsc_yakmo_seed_means(int n, int d, const float *x, int k, float *centroids);
int gsc_scan_reduce(int n, int d, const float *x, int k, float *centroids, int *clusters, int precision, int *iters);
/* -py reducer stage (cluster.py Birch labels, extern.pas:350-437): n x d
 * Single features of one frame -> labels[n] in [0, k). */
int gsc_birch_labels(int n, int d, const float *x, int k, int *labels);
int gsc_knnfit_assign(int r, int cs, const float *cand_fwd, int n, const float *q, float eps, int *best);
/* yakmo's prefix-chain fast path (gsc_yakmo.hip chain_fast, ppl = 8 or 16
 * points per lane) on 64*nbk points from *run: the accepted block count, the
 * run after them, and per accepted block the checkpoint / min / max of the
 * running f32 total (the DLL's sequential cum[], App. C.1).  Parity tests. */
int gsc_yakmo_chain_test(int ppl, const float *pts, int nbk, float run, int *accepted, float *run_out, float *ck,
                         float *bmn, float *bmx);

/* Timing of the last gsc_encode_* call on the calling thread (milliseconds),
 * split per stage, plus average device time per launch of each kernel. */
typedef struct {
    double host_prepare_ms, host_frames_ms, gpu_yakmo_ms, gpu_scan_ms, gpu_knnfit_ms, host_post_ms, total_ms;
    int frames, reduce_frames;
    long long points, scan_passes, scan_slow;
    long long scan_point_passes; /* sum over frames of passes * N (searches) */
    long long knnfit_pairs;      /* sum over frames of N * 4R (query x candidate) */
    int scan_launches, knnfit_launches;
    long long scan_restarts;     /* batched KNNScanReduce pipeline restarts */
    double gpu_dsp_ms;           /* device DSP incl. sample upload (attenuation divider, features) */
    double post_overlap_ms;      /* KNNFit + prune/sort + packing run while other frames were still scanning */
    int post_groups;             /* frame groups the post-processing pipeline ran */
    double gpu_recon_ms;         /* gsc_encode_wav_recon only: reconstruction + PsyADelta sum */
    long long knnfit_overflow;   /* queries whose tie set exceeded the 64-NN bucket (ANN replay) */
} gsc_timing;
void gsc_last_timing(gsc_timing *t);

int gsc_device_count(void);
/* bind the calling thread to a HIP device (one process per GPU) */
int gsc_set_device(int device);
const char *gsc_last_error(void);
void gsc_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
