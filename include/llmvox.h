/*
 * llmvox.h — C ABI of the MI355X-native LLMVoX streaming-TTS hot path
 * (libllmvox_hip.so, built for gfx950).
 *
 * The reference has no native boundary: its hot path is reached through the
 * duck-typed ModelHandler members that streaming_server.audio_generator_sync
 * calls (reference: streaming_server.py:250-426, inference/model_handler.py:45-166).
 * Each entry point below replaces one of those calls; the Python shim
 * (llmvox_amd/handler.py) binds them with ctypes and keeps the reference
 * signatures.
 *
 * Conventions
 *   - Every function returns 0 on success, a negative LVX_E* code on error;
 *     lvx_last_error() gives the message of the calling thread's last error.
 *   - Pointers named *_dev are device pointers on the context's device
 *     (e.g. torch tensor .data_ptr()); *_host are host pointers.
 *   - `stream` is a hipStream_t passed as void* (NULL = legacy default stream).
 *     All compute calls are asynchronous on that stream.
 *   - Layouts are row-major, dtypes are fixed per argument (float32 / int32 /
 *     int64) as named.
 */
#ifndef LLMVOX_H
#define LLMVOX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LVX_OK 0
#define LVX_E_ARG (-1)      /* bad argument / shape (reference: ValueError) */
#define LVX_E_STATE (-2)    /* weights missing / not finalized */
#define LVX_E_HIP (-3)      /* HIP runtime error */
#define LVX_E_CAPACITY (-4) /* position >= block_size or KV capacity (reference: AssertionError,
                               src/model.py:205) */
#define LVX_E_NAME (-5)     /* unknown weight name */
#define LVX_E_INDEX (-6)    /* an embedding id out of range, reported by lvx_check_errors (reference:
                               IndexError from nn.Embedding / the codebook gather) */

#define LVX_DTYPE_F32 0
#define LVX_DTYPE_BF16 1
#define LVX_DTYPE_FP8 2 /* kv_dtype: OCP e4m3fn (the gfx950 format), saturating at +-448, unscaled;
                           codec_dtype: e4m3fn codec GEMM weights with one fp32 scale per output row */

typedef struct lvx_ctx lvx_ctx;

typedef struct {
  int device;           /* HIP device ordinal */
  int weight_dtype;     /* LVX_DTYPE_F32 (parity mode; the reference runs fp32) or LVX_DTYPE_BF16 */
  int kv_dtype;         /* LVX_DTYPE_F32, LVX_DTYPE_BF16 or LVX_DTYPE_FP8 */
  int max_streams;      /* KV slots (concurrent utterance streams) */
  int max_positions;    /* per-slot KV capacity, <= 8192 (GPTConfig.block_size) */
  int max_codec_frames; /* max sum over streams of frames per codec call */
  int codec_dtype;      /* codec conv / linear weight storage: 0 = weight_dtype, or LVX_DTYPE_FP8 (needs
                           weight_dtype BF16: fp8 weights, bf16 operands, fp32 accumulation) */
} lvx_config;

/* ---- lifetime ----------------------------------------------------------- */
int lvx_create(const lvx_config* cfg, lvx_ctx** out);
/* replaces ModelHandler.__init__'s device placement (model_handler.py:48-63) */
void lvx_destroy(lvx_ctx* ctx);
const char* lvx_last_error(void);
int lvx_version(void);

/* ---- weights (by reference state_dict key, fp32 host data) -------------
 * replaces initialize_gpt_model / initialize_wavtokenizer / initialize_llm_model
 * (model_handler.py:66-78,80-106,140-166). Keys: "transformer.*", "lm_head.weight",
 * "backbone.*", "head.out.*", the codebook
 * "feature_extractor.encodec.quantizer.vq.layers.0._codebook.embed", and
 * "encoder.embed_tokens.weight" (the [386,256] text table). */
int lvx_set_weight(lvx_ctx* ctx, const char* name, const float* data_host, int64_t numel);
int lvx_finalize(lvx_ctx* ctx);
/* number of required weights not yet set; fills *first_missing (may be NULL) */
int lvx_missing_weights(lvx_ctx* ctx, const char** first_missing);

/* ---- text / code embeddings -------------------------------------------- */
/* ModelHandler.llm_model(ids): T5 encoder.embed_tokens gather
 * (streaming_server.py:315,319). ids int64 [n] -> out float32 [n,256]. An id outside [0, 386) is
 * clamped and flagged: the next lvx_check_errors returns LVX_E_INDEX (the same for codes outside
 * [0, 4096) in lvx_codes_to_features). */
int lvx_text_embed(lvx_ctx* ctx, const int64_t* ids_dev, int n, float* out_dev, void* stream);
/* WavTokenizer.codes_to_features (decoder/pretrained.py:209-239), n_q = 1:
 * codes int64 [B,L] -> features float32 [B,512,L] */
int lvx_codes_to_features(lvx_ctx* ctx, const int64_t* codes_dev, int B, int L, float* feats_dev,
                          void* stream);

/* ---- speech-token GPT ------------------------------------------------------ */
/* Forget a stream's KV (the reference sets kvcache = None, streaming_server.py:412). */
int lvx_stream_reset(lvx_ctx* ctx, int slot, void* stream);
/* GPT.forward(emb, kvcache) for one stream (src/model.py:201-237): emb_row_dev is the LAST
 * row of the caller's history (already normalised input, float32 [768]); pos is its index
 * t-1. Appends K/V at pos in slot `slot`, attends over [0, pos], writes logits float32
 * [4096]. */
int lvx_ar_forward_row(lvx_ctx* ctx, int slot, int pos, const float* emb_row_dev, float* logits_dev,
                       void* stream);
/* One fused decode step for B batch rows (a2..a11 of the hot path). Row b drives slot
 * slots[b] (-1 = idle row: computes nothing that is stored). With j = rowstep[b] and p the
 * slot's device-side position: input = normalize(cat(text_table[text_plan[b][j]],
 * p == 0 ? 0 : codebook[prev_token[slot]])) + wpe[p]  (streaming_server.py:325-338,
 * src/model.py:206-217); runs the 4 blocks, ln_f, lm_head and the greedy argmax (first
 * maximal index = argmax(softmax), streaming_server.py:342-346); writes tok_plan[b][j]
 * (and margin_plan[b][j] = top1 - top2 logit, optional), stores the token as the slot's
 * prev_token, advances the slot's position and rowstep[b]. text_plan / tok_plan /
 * margin_plan are [B][plan_stride] device arrays, so a whole chunk of steps can be enqueued
 * back to back (replayed as a HIP graph) and read back once. Inside a call the select of step i
 * is committed by the first kernel of step i + 1 (option "defer_select"); the last one by a
 * closing kernel of the call, so every output is in place when the call's work on `stream` is. */
int lvx_ar_step(lvx_ctx* ctx, int B, const int32_t* slots_dev, const int32_t* text_plan_dev,
                int plan_stride, int32_t* rowstep_dev, int32_t* tok_plan_dev, float* margin_plan_dev,
                void* stream);
/* n_steps consecutive lvx_ar_step calls with the same arguments. */
int lvx_ar_steps(lvx_ctx* ctx, int n_steps, int B, const int32_t* slots_dev, const int32_t* text_plan_dev,
                 int plan_stride, int32_t* rowstep_dev, int32_t* tok_plan_dev, float* margin_plan_dev,
                 void* stream);
/* Copy the logits [B][4096] of the last lvx_ar_step(s) call (diagnostics / tests). */
int lvx_ar_logits(lvx_ctx* ctx, int B, float* dst_dev, void* stream);
/* Synchronises the stream and reports (then clears) device-side errors of both error words: an embedding id or codec
 * code out of range (LVX_E_INDEX), the ISTFT window envelope <= 1e-11 (LVX_E_STATE; reference:
 * the assertion of decoder/spectral_ops.py:72 -- the fixed periodic Hann envelope is >= 0.72 on the
 * trimmed span, so this is a self-check), a slot past max_positions (LVX_E_CAPACITY; reference:
 * the block_size AssertionError, src/model.py:205) or a row past the end of its plan
 * (LVX_E_CAPACITY), or a non-finite / out-of-range (|v| >= 2^25) partial in the B <= 2 fused MLP's
 * fixed-point accumulation (LVX_E_STATE; the reference would carry the value into its logits). */
int lvx_check_errors(lvx_ctx* ctx, void* stream);
/* The device error bits live in two words: the AR word (decode steps, lvx_text_embed,
 * lvx_codes_to_features) and the codec word (lvx_codec_decode_*), so a codec running on a second stream
 * beside the decode keeps its flags apart. lvx_check_errors takes both; every condition that is set is
 * named in lvx_last_error (the code is the most specific one: LVX_E_INDEX > LVX_E_STATE >
 * LVX_E_CAPACITY). A take reads and clears the words atomically, in stream order: bits set later by
 * work in flight on another stream stay for the next take. */
#define LVX_ERRW_AR 1
#define LVX_ERRW_CODEC 2
/* Asynchronous take (no synchronisation): the bits of the chosen words (`which` = LVX_ERRW_AR and/or
 * LVX_ERRW_CODEC) into bits_dev[0] (device int32: AR bits | codec bits << 16), enqueued on `stream`
 * after the work already there; pass them to lvx_error_status once they are on the host. Lets a
 * scheduler read a chunk's errors with its tokens, without a stream synchronisation. */
int lvx_error_take(lvx_ctx* ctx, int which, int32_t* bits_dev, void* stream);
/* The status (and lvx_last_error message) of taken bits, as lvx_check_errors would return it; 0 if none. */
int lvx_error_status(int bits);
/* Set a slot's position and previous token (rewind after a speculative run-ahead, or jump). */
int lvx_stream_set(lvx_ctx* ctx, int slot, int pos, int prev_token, void* stream);
/* Measurement hook (bench.py): launch one kernel class of the decode step `iters` times for the
 * batch rows `slots` at their current positions (0 c_attn, 1 attention, 2 c_proj+merge,
 * 3 c_fc (with the bf16 fused MLP at B <= 2: c_fc + gelu + mlp c_proj), 4 mlp c_proj, 5 lm_head).
 * Writes only scratch and the K/V row at the current position (which the next real step
 * overwrites). LVX_E_STATE when the op has no kernel of its own at this B (fused). */
int lvx_probe_kernel(lvx_ctx* ctx, int which, int B, const int32_t* slots_dev, int iters, void* stream);
/* Test hook: the greedy select (argmax(softmax(logits)) with the reference's tie semantics,
 * streaming_server.py:342-346) of one production kernel path over caller-given logits float32
 * [B][4096], committed exactly as a decode step commits it (tok_plan[b][rowstep[b]], margin,
 * slot prev / position, rowstep advance). path 0: ar_argmax_kernel; 1: the lm_head-granule
 * reduction of the B <= 2 deferred select (B <= 4 here); 2: the batched deferred select
 * (ar_embed_select_kernel). plan_stride >= 2. */
int lvx_select_probe(lvx_ctx* ctx, int path, int B, const int32_t* slots_dev, const float* logits_dev,
                     const int32_t* text_plan_dev, int plan_stride, int32_t* rowstep_dev, int32_t* tok_plan_dev,
                     float* margin_plan_dev, void* stream);
/* Host-side view of a slot's position (synchronises the stream). */
int lvx_stream_position(lvx_ctx* ctx, int slot, int* pos_out, void* stream);
/* Cross-check switches between two correct implementations of the same step, per context (round 4:
 * an option set on one context never changes another context's kernels; each call binds a snapshot
 * of its context's options, and the context drops its captured graphs on its next call after a
 * change). Defaults are the measured-faster variants:
 *   "defer_select" 1: the greedy select is committed by the next step's first kernel (bf16 with "l0q"
 *                     1: ar_embed_select at every B; otherwise B <= 2 and 4 <= B <= 8: c_attn layer 0
 *                     reduces lm_head's granules, larger B: ar_embed_select); 2: 4 <= B <= 8 through
 *                     ar_embed_select with "l0q" 0 too; 0: ar_argmax_kernel after every lm_head
 *                     (bit-identical results with "l0q" 0: tests/test_gpu_select.py);
 *   "fuse_mlp"     1: bf16, B <= 2: c_fc + gelu + mlp c_proj in one kernel (2^-32 fixed-point int64
 *                     atomics: exact sums, reproducible run to run); 0: the two GEMV kernels;
 *   "bt"           1: batched path v3 for 32 < B <= 64; 2: v3 for every batched B; 0: never;
 *   "codec_g2"     1: large-M bf16 codec GEMMs on the 128 x 128 MFMA tile kernel; 0: the general one;
 *   "codec_skinny" 1: bf16 codec weight GEMMs with M <= 384 frames on the K-split-over-waves kernel
 *                     (no split-K combine); 0: the tile kernels;
 *   "codec_g3f"    fp32 (parity mode) codec GEMMs with >= 192 tiles of 128 x 192: 2 (default): the
 *                     LDS-DMA kernel with fp32 operands split into bf16 hi + lo, hi.hi + lo.hi + hi.lo
 *                     on v_mfma_f32_16x16x32_bf16 (fp32 accumulation); 1: the same kernel with exact-fp32
 *                     v_mfma_f32_16x16x4_f32 (slower; the tests' exact-fp32 oracle for the split form);
 *   "codec_exp"    codec development bits, 0 = production kernels; bit 0: the general GroupNorm
 *                     kernel at every L (same bits); bits 1-2: dwconv+AdaLN frames per block at
 *                     >= 2,048 frames (0: 4, 1: 16, 2: 32, 3: 8; same bits); bit 3: library
 *                     exp / sin / cos in the bf16 iSTFT; bit 4: fp32 bf16x3 GEMMs split their
 *                     operands in registers, no split-image producers (same bits);
 *   "exp"          cross-check bits, 0 = production kernels (fp32 parity mode, each bit-identical or
 *                     within fp32 summation noise: tests/test_gpu_f32b.py); bit 8: fp32 batched GEMMs
 *                     in 32-row instead of 16-row batch tiles (bit-identical); bit 512: fp32 mlp c_proj
 *                     unsplit, bit 1024: fp32 c_attn in one launch (another summation order);
 *   "f32b"         1: fp32 weights, 3 <= B <= 64: batched steps on exact-fp32 MFMA (ar_f32b_kernel);
 *                     0: the fp32 GEMV family (same ids against the reference: tests/test_gpu_f32b.py);
 *   "ln_max"       (2..8, default 8) largest B whose batched GEMMs normalise in their own prologue;
 *                  larger B run the rows kernel + batched GEMM structure;
 *   "l0q"          1: bf16 weights, B <= 32 (not 3) with the deferred select: layer 0's c_attn from
 *                     table rows precomputed at lvx_finalize (text / codebook / position x ln_1 x W),
 *                     inside the embedding + select kernel (B > 8: one launch less per step; B <= 8:
 *                     the step's first launch reads three table rows instead of weight slices; the
 *                     operand is not rounded to bf16, so the sums differ from the GEMM's in the last
 *                     bits: tests/test_gpu_batched.py, test_gpu_select.py); 0: the c_attn GEMM / GEMV
 *                     (B > 8 after the embedding + select kernel; B <= 8 with the granule select). */
int lvx_set_option(lvx_ctx* ctx, const char* name, int value);
/* The stream the decode graphs are captured on (then replayed on the caller's stream). NULL (default):
 * the caller's stream. Name another one when something may query, from another thread, an event
 * recorded on the caller's stream while lvx_ar_step* runs (a process group's watchdog after a
 * synchronous collective on that stream): HIP refuses such a query during a capture. The stream
 * named must not be the caller's and must outlive the context's use of it. */
int lvx_set_capture_stream(lvx_ctx* ctx, void* stream);
/* Enable/disable HIP-graph replay of lvx_ar_step for a given B (default on). */
int lvx_set_graphs(lvx_ctx* ctx, int enable);

/* ---- codec decoder ------------------------------------------------------- */
/* WavTokenizer.decode(features, bandwidth_id) (decoder/pretrained.py:192-207):
 * features float32 [B,512,L] (the reference layout) -> pcm float32 [B, 320*L]. Streams are
 * decoded independently (each one exactly as a separate reference call with its own L). */
int lvx_codec_decode_features(lvx_ctx* ctx, const float* feats_dev, int B, int L, int bandwidth_id,
                              float* pcm_dev, void* stream);
/* codes_to_features + decode fused: codes int32 [B,L] -> pcm float32 [B,320*L]. A code outside
 * [0, 4096) is clamped for the gather and flagged (the next lvx_check_errors: LVX_E_INDEX). */
int lvx_codec_decode_codes(lvx_ctx* ctx, const int32_t* codes_dev, int B, int L, int bandwidth_id,
                           float* pcm_dev, void* stream);

/* ---- WavTokenizer encoder, a context of its own (its weights are not needed for TTS).
 * Replaces WavTokenizer.encode_infer (WavTokenizer/decoder/pretrained.py:185-190 ->
 * decoder/feature_extractors.py:122-133): SEANet encoder (encoder/modules/seanet.py:94-143) + the
 * 1-codebook quantiser (encoder/quantization/vq.py:115-140, core_vq.py:175-183), fp32.
 * Weights by reference state_dict name: "feature_extractor.encodec.encoder.model.<i>.conv.conv.weight"
 * with weight_norm already resolved (w = g v / |v|, torch._weight_norm(v, g, 0)) [cout][cin][k], ".bias",
 * the LSTM's "<...>.13.lstm.{weight,bias}_{ih,hh}_l{0,1}", and the codebook
 * "feature_extractor.encodec.quantizer.vq.layers.0._codebook.embed" [4096][512]. */
typedef struct lvx_enc lvx_enc;
int lvx_enc_create(int device, long long max_samples, lvx_enc** out);  /* max_samples >= B * N of any call */
int lvx_enc_set_weight(lvx_enc* enc, const char* name, const float* data, int64_t numel);
int lvx_enc_finalize(lvx_enc* enc);
void lvx_enc_destroy(lvx_enc* enc);
/* frames T of an N-sample input (ceil(N / 320): the SConv1d padding chain) */
int lvx_enc_frames(int n_samples);
/* audio_dev [B][N] f32 -> features_dev [B][512][T] (codebook rows of the codes, the reference's
 * features layout), codes_dev [B][T] int32 (the reference returns them as [1][B][T]). Async on stream. */
int lvx_encode(lvx_enc* enc, const float* audio_dev, int B, int N, float* features_dev, int32_t* codes_dev,
               void* stream);
/* test hook: the pre-quantisation embedding [B][T][512] of the last lvx_encode */
int lvx_enc_embedding(lvx_enc* enc, float* dst_dev, int B, int T, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LLMVOX_H */
