/*
 * tonehip.h -- C ABI of libtonehip.so, the MI355X-native T-one streaming acoustic path.
 *
 * This is the boundary that replaces ONNX Runtime under tone/onnx_wrapper.py:
 *
 *   reference                                             | this library
 *   ------------------------------------------------------+------------------------------------
 *   ort.InferenceSession(model_path, providers=...)       | tone_session_create + tone_session_set_weight
 *     (tone/onnx_wrapper.py:76-78)                        |   (one call per checkpoint tensor) + tone_session_finalize
 *   ort_sess.run(None, {"signal": chunk, "state": state}) | tone_session_run
 *     (tone/onnx_wrapper.py:123; I/O names and dims:      |   signal (B,2400,1) int32, state (B,219729) fp16
 *      configs/streaming_acoustic/config.pbtxt:5-33)      |   -> logprobs (B,10,35) fp32, state_next (B,219729) fp16
 *   Triton sequence batching with server-side state       | tone_session_run_slots (device-resident state slab,
 *     (triton/model/config.pbtxt:26-69)                   |   stream slots gathered by index)
 *
 * All tensor arguments are DEVICE pointers (HIP global memory on the session's device); no torch
 * types cross the boundary.  Every call is asynchronous on the given hipStream_t (passed as void*,
 * NULL = the legacy default stream).  Functions return 0 on success or a negative TONE_E_* code;
 * tone_last_error() returns a thread-local description of the last failure.
 *
 * A session is not re-entrant: serialize calls on one session (one session per GPU / per thread).
 */
#ifndef TONEHIP_H
#define TONEHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TONE_ABI_VERSION 1

/* boundary constants, tone/onnx_wrapper.py:30-34 */
#define TONE_SAMPLE_RATE 8000
#define TONE_AUDIO_CHUNK_SAMPLES 2400
#define TONE_STATE_SIZE 219729
#define TONE_FRAMES_PER_CHUNK 10
#define TONE_VOCAB 35

/* precision of the dense contractions; everything else (norms, softmax, log-softmax, state
 * arithmetic) is fp32 in every mode, and the state is fp16 at the boundary. */
#define TONE_PRECISION_FP32 0      /* fp32 GEMMs as exact 3-way bf16 splits (6 products, fp32 accumulate) */
                                   /* on v_mfma_f32_32x32x16_bf16: fp32-accurate, BASELINE config 2      */
#define TONE_PRECISION_BF16 1      /* bf16 MFMA operands, fp32 accumulate, BASELINE config 3            */
#define TONE_PRECISION_FP32_MFMA 2 /* fp32 GEMMs on the exact-fp32 MFMA (v_mfma_f32_32x32x2_f32)       */
#define TONE_PRECISION_FP8 3       /* bf16 mode, with the q/k/v and FFN GEMMs on MXFP8 (e4m3 values, one */
                                   /* E8M0 scale per 32 along K) on v_mfma_scale_f32_16x16x128_f8f6f4:   */
                                   /* BASELINE config 5                                                   */

#define TONE_OK 0
#define TONE_E_INVALID -1   /* bad argument (shape, null pointer, unknown name)       */
#define TONE_E_STATE -2     /* call out of order (run before finalize, ...)          */
#define TONE_E_HIP -3       /* a HIP runtime call failed                             */
#define TONE_E_MISSING -4   /* finalize with checkpoint tensors missing              */

typedef struct tone_session tone_session;

int tone_abi_version(void);
const char *tone_last_error(void);

/* Create a session on `device` able to run batches of up to `max_batch` streams. */
int tone_session_create(tone_session **out, int device, int precision, int max_batch);
int tone_session_destroy(tone_session *s);

/* Provide one checkpoint tensor by its reference state_dict name (tone/nn/model.py:39-41,
 * e.g. "encoder.layers.3.feed_forward1.linear1.weight"; an HF "tone." prefix is accepted), as
 * host fp32 data of exactly the reference shape's element count. */
int tone_session_set_weight(tone_session *s, const char *name, const float *host_data, int64_t numel);

/* Fold (RMSNorm gains into the following GEMM, BatchNorm into the preceding conv), pack
 * (SwiGLU/GLU pairs interleaved, q|k|v concatenated) and upload the weights. */
int tone_session_finalize(tone_session *s);

/* Chunk length of the session's steps, before tone_session_finalize: 2400 samples (300 ms, default;
 * tone/onnx_wrapper.py:32 AUDIO_CHUNK_SAMPLES) or 3200 (400 ms: the Triton ensemble's chunk,
 * triton/ensemble/config.pbtxt:12-18; tone/scripts/export.py:139-157 chunk_duration_ms).  The flat state
 * layout is the same; a 400 ms step reads signal [batch][3200] and writes logprobs [batch][13][35]. */
int tone_session_set_chunk(tone_session *s, int chunk_samples);
/* Acoustic frames per step: 10 (300 ms) or 13 (400 ms). */
int tone_session_frames_per_chunk(const tone_session *s);

/* Enable (1) / disable (0) hipGraph capture+replay of the per-step kernel sequence, keyed by
 * (batch, I/O pointers, frame_info pointer, state stride).  At most 16 executable graphs are kept
 * (least recently used evicted), so callers should reuse fixed I/O buffers.  Runs on the NULL stream,
 * with timing on, or with a debug stop set are never captured.  Default 0. */
int tone_session_set_graph(tone_session *s, int enable);

/* Optional per-frame decode outputs of later runs (device pointer, int32 [batch][frames], or NULL):
 *   frame_info = greedy CTC token (argmax over 35, first index on ties; tone/decoder.py:57)
 *              | speech flag << 8 (exp(lp[33]) + exp(lp[34]) <= 0.9; tone/logprob_splitter.py:134)
 * computed in the head kernel from the logprobs it writes.  Replaces the host-side argmax and
 * threshold of GreedyCTCDecoder / StreamingLogprobSplitter (10 ids + 10 bits per stream-chunk). */
int tone_session_set_frame_info(tone_session *s, int32_t *frame_info);

/* One streaming step for `batch` independent streams.
 *   signal      int32  [batch][2400 | 3200]   PCM, int16 range (validated by the caller)
 *   state_in    fp16   [batch][state_stride]  first 219729 elements are the flat state
 *   logprobs    fp32   [batch][10 | 13][35]   (tone_session_frames_per_chunk)
 *   state_out   fp16   [batch][state_stride]  must not alias state_in
 * state_stride >= 219729 (elements). */
int tone_session_run(tone_session *s, const int32_t *signal, const uint16_t *state_in, float *logprobs,
                     uint16_t *state_out, int batch, int64_t state_stride, void *stream);

/* Same step with the state in a device-resident slab of n_slots rows: stream i reads row
 * slots[i] of slab_in and writes row slots[i] of slab_out.
 *   slots       int32  [batch]                device memory; ids distinct and in [0, n_slots) -- the
 *                                             kernels index the slabs with them unchecked, so the caller
 *                                             validates (tone_amd.model.ToneSession.run_slots does)
 *   slab_in/out fp16   [n_slots][slab_stride] slab_stride >= 219729, equal for both, not aliased
 * Rows of slab_out not named in slots are not written. */
int tone_session_run_slots(tone_session *s, const int32_t *signal, const int32_t *slots, const uint16_t *slab_in,
                           uint16_t *slab_out, int64_t slab_stride, float *logprobs, int batch, void *stream);

/* Same step over ONE slab whose rows are used in ping-pong: stream i reads row rows_in[i] and writes
 * row rows_out[i] (device int32 [batch] each).  No row may appear in both lists, and the ids must be
 * in [0, n_rows) (unchecked, as for run_slots).  A server keeps two rows per stream and flips only the
 * streams that step, so streams without audio this step keep their state with no copy. */
int tone_session_run_rows(tone_session *s, const int32_t *signal, const int32_t *rows_in, const int32_t *rows_out,
                          uint16_t *slab, int64_t slab_stride, float *logprobs, int batch, void *stream);

/* Same step with the state in its RESIDENT form: the conv-module caches and the layer 14 / 15 MHSA input caches (the
 * (16, 384, 30) and (2, 30, 384) sections, 94 % of the 439 KB state) live outside the rows in one ring per stream,
 * updated in place -- a step reads the cached frames and writes only its T new ones over the T oldest, where the flat
 * form rewrites the whole window shifted by T.
 *   rows_in/out int32 [batch]                     ping-pong rows of `slab` for the other sections (as run_rows)
 *   rings       fp16  [n_rings][tone_session_ring_elems()]   time-major [16 + 2][30][384]
 *   ring_ids    int32 [batch]                     stream i's ring (distinct, in [0, n_rings), unchecked)
 * The row's conv section then holds only the stream's chunk counter (mod 30), which sets the rings' phases; its mhsa
 * section is unused.
 * Results (logprobs, and the state once exported) are bit-identical to the flat form's.  Convert with
 * tone_session_ring_import (flat row i -> slab row rows[i] + ring ring_ids[i]; a zero flat state gives a fresh stream)
 * and tone_session_ring_export (the inverse: the flat (B, 219729) state at the boundary). */
int tone_session_run_ring(tone_session *s, const int32_t *signal, const int32_t *rows_in, const int32_t *rows_out,
                          uint16_t *slab, int64_t slab_stride, uint16_t *rings, const int32_t *ring_ids, float *logprobs,
                          int batch, void *stream);
int tone_session_ring_import(tone_session *s, const uint16_t *flat, int64_t flat_stride, uint16_t *slab,
                             int64_t slab_stride, const int32_t *rows, uint16_t *rings, const int32_t *ring_ids, int n,
                             void *stream);
int tone_session_ring_export(tone_session *s, const uint16_t *slab, int64_t slab_stride, const int32_t *rows,
                             const uint16_t *rings, const int32_t *ring_ids, uint16_t *flat, int64_t flat_stride, int n,
                             void *stream);
/* fp16 elements of one stream's ring ((16 + 2) x 30 x 384). */
int64_t tone_session_ring_elems(void);

/* Workspace bytes the session holds on the device (weights + activations). */
int64_t tone_session_device_bytes(const tone_session *s);

/* Average duration in microseconds of the named kernel family over the last timed run
 * (see tone_session_set_timing); used by bench.py for the roofline figure. */
int tone_session_set_timing(tone_session *s, int enable);
double tone_session_kernel_us(const tone_session *s, const char *family, int64_t *launches);

/* ---- diagnostics (parity localisation; not needed for serving) ------------------------------
 * tone_session_debug_stop: end the step early -- stage 0 after the log-mel front end, 1 after the
 * subsampling (pre-encode + out_norm), 2 + L after Conformer layer L (incl. reduction/upsampling
 * at L = 6 / 14), 100 + L after layer L's pw2 (fp8: FFN2's MXFP8 operand made); -1 (default) runs
 * the whole step.  Requires graph mode off.
 * tone_session_debug_read: copy an internal buffer of the last step to host memory: fp32 activations
 * ("feats", "x2", "flat", "rA", "rB"), fp8 mode's next MX GEMM operand ("a8" e4m3 [rows][384], "a8s"
 * E8M0 [rows][12], "ss8" fp32 sum-of-squares slab [rows][12]). */
int tone_session_debug_stop(tone_session *s, int stage);
int tone_session_debug_read(tone_session *s, const char *buffer, void *host_dst, int64_t bytes);

#ifdef __cplusplus
}
#endif

#endif /* TONEHIP_H */
