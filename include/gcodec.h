/*
 * gcodec.h — C ABI of libgcodec, the MI355X-native (gfx950) QSGD-MaxNorm
 * gradient codec.
 *
 * Plain C: raw pointers, sizes and an opaque stream handle; no torch or HIP
 * types.  Every device entry point takes caller-owned device buffers, never
 * allocates, never synchronises the host, and enqueues on `stream` (a
 * hipStream_t passed as void*; NULL = the legacy default stream), so a call
 * sequence is hipGraph-capturable.  Status: 0 = GC_OK, negative = error;
 * gc_last_error() returns a thread-local description of the last failure.
 *
 * Reference interfaces each entry point replaces (vineeths96/
 * Gradient-Compression; file:line):
 *   gc_absmax_f32 ............ reducer.py:516,726,1478,1577,1663  buffer.abs().max()
 *   gc_qsgd_encode ........... compressors.py:299-316 QSGDMaxNormCompressor.compress
 *                              (+ GlobalRandKMaxNormCompressor.compress 435-451 with idx)
 *                              fused with the packing intent of compressors.py:357-358 /
 *                              extensions/Extension CPU/bitpacking.cpp:5-61 (carry-free lanes)
 *   gc_qsgd_decode ........... compressors.py:318-321 decompress (+ reducer.py:549 alpha=1/W,
 *                              + reducer.py:754 scatter with idx)
 *   gc_randk_* ............... reducer.py:722-735 GlobalRandK gather buffer[idx] + its max-norm
 *                              (+ compressors.py:435-451 compress, fused at W = 1)
 *   gc_qsgd_quantize ......... compressors.py:299-316, unpacked int8/int32 output (literal drop-in)
 *   gc_qsgd_dequantize ....... compressors.py:318-321, unpacked input
 *   gc_qsgd_quantize_split ... compressors.py:338-353 QSGDBPCompressor.compress (sign bits + xi)
 *   gc_lane_pack/_unpack ..... extensions/Extension GPU/gpu_bitpacking.cpp:5-125 intent
 *                              (device packing of quantized ints), sum-compatible format
 *   gc_ms_mask_encode ........ compressors.py:778-807 compress_cache + compress_mask
 *                              (= TwoScale compress_lower/compress_higher 630-666 for 2 levels)
 *   gc_ms_select_encode ...... compressors.py:809-817 compress(mask) (+ reducer.py:1503-1505 blend)
 *   gc_ms_encode_w1 .......... both at W = 1 (reducer.py:1680 MIN over one rank = identity), one pass
 *   gc_ms_*_cached ........... the same pair with compressors.py:778-797's cache kept (packed cells)
 *   gc_ms_decode ............. compressors.py:819-826 (order 0) / 668-680 (order 1)
 *   gc_mt19937_seed/_generate  seed.py:6-11 torch.manual_seed + torch CPU generator stream
 *   gc_mt19937_*jump*          consumed by torch.bernoulli (compressors.py:310); the
 *                              jumped form generates it in parallel
 *   gc_greedy4_pack/_unpack .. extensions/Extension CPU/bitpacking.cpp:5-124 (host, same format)
 *   gc_greedy4_*_device ...... the same format on the device (Extension GPU/gpu_bitpacking.cpp:5-125
 *                              is host code despite its name; this is the GPU drop-in)
 *   gc_bytepack8/_unpack8 .... extensions/Extension CPU BP/bytepacking.cpp:6-64 (device)
 *   gc_segments_* ............ reducer.py:46-68 TensorBuffer (flatten / views) and the setgrad
 *                              loop reducer.py:543-549 (+ 753-761, 1521-1527, 1705-1711):
 *                              fused flatten + max-norm, decode straight into the per-parameter
 *                              gradients, and the scaled scatter of a flat bucket
 */
#ifndef GCODEC_H
#define GCODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GC_ABI_VERSION 1

/* status codes */
#define GC_OK 0
#define GC_EINVAL (-1)  /* bad argument (null pointer, bits, layout mismatch) */
#define GC_EHIP (-2)    /* HIP runtime / launch error */
#define GC_ERANGE (-3)  /* value outside the format's domain (greedy4: <0 or >255) */
#define GC_ENOSPC (-4)  /* output capacity too small */
#define GC_ENODEV (-5)  /* no gfx950 device */

/* element dtypes for the unpacked-integer entry points */
#define GC_I8 1u
#define GC_I32 4u
#define GC_I64 8u

/* random streams for the stochastic rounding */
#define GC_RNG_PHILOX 0u /* Philox4x32-10 keyed by seed, counter (element>>2, level, offset) */
#define GC_RNG_STREAM 1u /* caller-supplied 32-bit draws, level-major: stream[level*n + i] */
/* caller-supplied draws packed to their low 24 bits, 3 bytes each, little-endian
 * (element i at bytes 3i .. 3i+2; the rounding reads only those bits), one
 * level: gc_qsgd_encode only (the torch-mode encode's draws from
 * gc_mt19937_generate_split24_j); stream 4-byte aligned */
#define GC_RNG_STREAM24 2u
/* caller-supplied draws cut into two planes (torch-mode encode): of draw i's
 * low 24 bits, the top hb bits (hb = 8: SPLIT8, 16: SPLIT16) in the HI plane
 * (hb/8 bytes per draw, little-endian) and the rest in the LO plane, which
 * starts at stream + roundup(n * hb/8, 16) bytes; gc_rng_split_bytes(n, hb)
 * bytes in all.  The encode reads the LO plane only for the quads whose HI
 * bits leave the rounding undecided (about 1 draw in 2^hb).  One level:
 * gc_qsgd_encode only; stream 16-byte aligned (gc_mt19937_generate_multi_split_j) */
#define GC_RNG_SPLIT8 3u
#define GC_RNG_SPLIT16 4u

typedef void *gc_stream_t; /* hipStream_t */

typedef struct gc_rng {
    uint32_t kind;          /* GC_RNG_PHILOX | GC_RNG_STREAM | GC_RNG_STREAM24 | GC_RNG_SPLIT8 | GC_RNG_SPLIT16 */
    uint32_t reserved;      /* 0 */
    uint64_t seed;          /* PHILOX key */
    uint64_t offset;        /* PHILOX: draws consumed before this call (counter high words) */
    const uint32_t *stream; /* STREAM: device pointer to the draws */
} gc_rng;

/* Carry-free planar lane layout of a packed stream.
 * Each element contributes a lane value in [0, range] (offset binary:
 * lane = q + offset).  Lanes are `bits` wide with bits = bit_length(world*range),
 * so a SUM all-reduce of the uint32 words over `world` ranks never carries
 * between lanes.  per_word = floor(32/bits) lanes per word.  Planar: word j
 * holds elements j, j+M, ..., j+(per_word-1)*M, M = plane_words =
 * roundup(ceil(n/per_word), A), A = 64 words if ceil(n/per_word) >= 65536 else 4.
 * Elements >= n contribute 0 bits. */
typedef struct gc_lanes {
    uint64_t n;           /* elements */
    uint64_t plane_words; /* M = words in the stream */
    uint32_t bits;        /* lane width w */
    uint32_t per_word;    /* L */
    uint32_t offset;      /* lane = q + offset */
    uint32_t world;       /* W the lanes were sized for */
    uint64_t range;       /* per-rank lane value range [0, range] */
} gc_lanes;

/* ascending quantization levels (bits) of the multi-scale codec */
#define GC_MAX_LEVELS 8
typedef struct gc_levels {
    uint32_t count;
    uint32_t bits[GC_MAX_LEVELS];
} gc_levels;

/* ---- library ---------------------------------------------------------- */
const char *gc_version(void);
const char *gc_last_error(void);
int gc_abi_version(void);
int gc_device_check(int device); /* GC_OK if `device` is a gfx950 GPU */

/* ---- layouts (host, pure) ---------------------------------------------- */
int gc_lane_layout(uint64_t n, uint64_t range, uint32_t world, uint32_t offset, gc_lanes *out);
/* QSGD lanes: range 2s, offset s, s = 2^bits-1 */
int gc_qsgd_layout(uint64_t n, uint32_t bits, uint32_t world, gc_lanes *out);
/* multi-scale q lanes: qmax = s_0 (2 levels) or s_0+1 (>=3 levels) */
int gc_ms_layout(uint64_t n, const gc_levels *levels, uint32_t world, gc_lanes *out);
/* multi-scale mask lanes: (count-1) thermometer fields of range 1, each its own
 * stream of plane_words; total words = (count-1)*plane_words.
 * At world = 1 the two layouts are coupled: r = floor(32 / q per_word), the q
 * plane_words is a multiple of 64 r and the mask plane_words = q plane_words / r
 * (mask plane h + r k = q lane k of q words [h M_mask, (h+1) M_mask)), which
 * gc_ms_encode_w1 needs.  Every entry point accepts any plane_words at or
 * above the minimal layout's with its alignment. */
int gc_ms_mask_layout(uint64_t n, const gc_levels *levels, uint32_t world, gc_lanes *out);

/* ---- max-norm ----------------------------------------------------------- */
/* *norm = max_i |x[idx ? idx[i] : i]| over i < n (NaN-propagating); norm is a
 * device float overwritten by the call.  workspace: NULL (a memset of *norm
 * is enqueued first) or gc_absmax_workspace_size() device bytes, zeroed ONCE
 * by the caller and then reused (self-resetting; one workspace per stream).
 * Hardware assumption of the workspace form: every block stores its partial
 * with an sc1 (agent-coherent, write-through) store, drains it (s_waitcnt
 * vmcnt(0)) and only then takes a relaxed agent-scope ticket of its group
 * (block mod 16); each group's last block then takes a top-level ticket, and
 * the block that draws the last of those reads the partials with sc1 loads.
 * This is the fence-free hand-off MI355X_MICROARCH.md measures on gfx950,
 * not an ordering the HIP memory model promises for relaxed atomics (a
 * release/acquire pair emits an L2 write-back that doubles the kernel's
 * time; lib/libgcodec_strict.so is the build with that pair,
 * tests/test_gpu_strict_handoff.py).  tests/test_gpu_parity.py::
 * test_absmax_workspace_reuse_many_grids pins it over 1..512-block grids. */
size_t gc_absmax_workspace_size(void);
int gc_absmax_f32(const float *x, const int64_t *idx, uint64_t n, float *norm, void *workspace,
                  gc_stream_t stream);

/* ---- QSGD-MaxNorm ------------------------------------------------------- */
/* words[lanes->plane_words] = pack(q + s), q = stochastic_round(x[idx?idx[i]:i], *norm, bits) */
int gc_qsgd_encode(const float *x, const int64_t *idx, uint64_t n, const float *norm, uint32_t bits,
                   const gc_lanes *lanes, const gc_rng *rng, uint32_t *words, gc_stream_t stream);
/* out[idx?idx[i]:i] = RN(RN(RN(*norm/s) * (lane_sum - W*s)) * alpha) */
int gc_qsgd_decode(const uint32_t *words, const int64_t *idx, uint64_t n, const float *norm, uint32_t bits,
                   const gc_lanes *lanes, float alpha, float *out, gc_stream_t stream);
/* unpacked: q[i] (GC_I8 | GC_I32, wraps like torch .to()) for draw block `level` */
int gc_qsgd_quantize(const float *x, uint64_t n, const float *norm, uint32_t bits, const gc_rng *rng,
                     uint32_t level, void *q, uint32_t q_dtype, gc_stream_t stream);
/* as gc_qsgd_quantize; also le_mask[i] = (|q[i]| <= 2^le_bits - 1) computed on the
 * unwrapped magnitude — compressors.py:660 higher_resolution_mask of compress_higher */
int gc_qsgd_quantize_le(const float *x, uint64_t n, const float *norm, uint32_t bits, const gc_rng *rng,
                        uint32_t level, void *q, uint32_t q_dtype, int8_t *le_mask, uint32_t le_bits,
                        gc_stream_t stream);
/* the QSGDBP call site (compressors.py:338-353): xi[i] = stochastic_round(|x[i]| / *norm * s)
 * and sign[i] = 1 iff x[i] < 0 (0 for +-0), two int32 arrays — the inputs the
 * reference hands to its greedy packer (bitpacking.packing, compressors.py:357-358) */
int gc_qsgd_quantize_split(const float *x, uint64_t n, const float *norm, uint32_t bits, const gc_rng *rng,
                           int32_t *xi, int32_t *sign, gc_stream_t stream);
/* out[i] = RN(RN(RN(*norm/s) * q[i]) * alpha) */
int gc_qsgd_dequantize(const void *q, uint32_t q_dtype, uint64_t n, const float *norm, uint32_t bits,
                       float alpha, float *out, gc_stream_t stream);

/* ---- lane packing of already-quantized integers -------------------------- */
int gc_lane_pack(const void *q, uint32_t q_dtype, const gc_lanes *lanes, uint32_t *words, gc_stream_t stream);
/* q[i] = lane - world*offset (the W-way sum) */
int gc_lane_unpack(const uint32_t *words, const gc_lanes *lanes, int32_t *q, gc_stream_t stream);

/* ---- small-K GlobalRandK (reducer.py:717-754, compressors.py:419-456) -------
 * One element per thread over ceil(k/1024) blocks: xk[i] = x[idx[i]] (the subset,
 * contiguous) and *norm = max |xk| in one launch (the last block to finish reduces
 * the partials; workspace: gc_randk_workspace_size() device bytes zeroed once,
 * self-resetting, one per stream).  k <= 262144.  At W > 1 the encode then runs
 * on xk after the MAX all-reduce (gc_qsgd_encode, dense): the subset is gathered
 * once.  gc_randk_encode_w1 is the W = 1 step (the MAX over one rank is the
 * identity): gather + max-norm + quantize + pack in ONE launch, words identical to
 * gc_qsgd_encode(x, idx, ...) with lanes = gc_qsgd_layout(k, bits, 1); k <= 16384.
 * The decode-scatter is gc_qsgd_decode with idx. */
size_t gc_randk_workspace_size(void);
int gc_randk_gather_absmax(const float *x, const int64_t *idx, uint64_t k, float *xk, float *norm, void *workspace,
                           gc_stream_t stream);
int gc_randk_encode_w1(const float *x, const int64_t *idx, uint64_t k, float *xk, float *norm, uint32_t bits,
                       const gc_lanes *lanes, const gc_rng *rng, uint32_t *words, void *workspace, gc_stream_t stream);
/* the same two with x given as the per-parameter tensors (a gc_segments table,
 * below): the reducer's gather reads every index from its tensor, so no
 * flattened bucket is built for GlobalRandK (reducer.py:713-723 flattens the
 * whole gradient, then gathers K of its elements).  Indices are not
 * range-checked on the device: every idx[i] must be in [0, segs->n) */
typedef struct gc_segments gc_segments;
int gc_randk_gather_absmax_segments(const gc_segments *segs, const int64_t *idx, uint64_t k, float *xk, float *norm,
                                    void *workspace, gc_stream_t stream);
int gc_randk_encode_w1_segments(const gc_segments *segs, const int64_t *idx, uint64_t k, float *xk, float *norm,
                                uint32_t bits, const gc_lanes *lanes, const gc_rng *rng, uint32_t *words,
                                void *workspace, gc_stream_t stream);

/* ---- greedy 4-mode packer on the device --------------------------------------
 * The format of gc_greedy4_pack (Extension CPU/bitpacking.cpp:5-124) produced by
 * a parallel scan over 16-entry segment tables.
 * Results are asynchronous: *nwords / *count (device uint64) receive the
 * number of words / values, *status (device uint32) 0 or a bit set: 1 = a
 * value outside [0, 255], 2 = more than cap outputs, 4 = (pack) a block of the
 * persistent launch gave up waiting for the others (about a second).  With 1
 * or 2 set nothing is written when the pack runs in one round (n up to about
 * 25 M on 256 CUs); a longer pack has written the words of the rounds before
 * the one that found it.  The unpack writes nothing on 2.
 * workspace: gc_greedy4[_unpack]_workspace_size bytes, device.  The PACK
 * workspace must be zero-filled before its first use and is left that way by
 * every call (after status 4: zero it again); the unpack workspace needs no
 * initialisation.  One pack at a time per pack workspace, and one pack in
 * flight per DEVICE: the pack is persistent (one block per CU, each waiting
 * for every block of its launch), so two packs running at once on different
 * streams can hold the CUs each other's blocks need until both time out —
 * order packs on different streams with events.  Status 4 = some block
 * waited longer than ~1.3 s (every block's timeout is collected); the words
 * are then incomplete.  unpack emits whole words (the caller truncates, as
 * compressors.py:371 does). */
size_t gc_greedy4_workspace_size(uint64_t n);
int gc_greedy4_pack_device(const int32_t *src, uint64_t n, int32_t *out, uint64_t cap, uint64_t *nwords,
                           uint32_t *status, void *workspace, gc_stream_t stream);
size_t gc_greedy4_unpack_workspace_size(uint64_t nwords);
int gc_greedy4_unpack_device(const int32_t *words, uint64_t nwords, int32_t *out, uint64_t cap, uint64_t *count,
                             uint32_t *status, void *workspace, gc_stream_t stream);

/* ---- per-parameter tensors (the reference's TensorBuffer) ------------------
 * A gc_segments describes `count` contiguous fp32 tensors laid end to end as
 * one flat bucket of n elements (reducer.py:46-68): flat element e lives at
 * seg[s].ptr[e - seg[s].start] for the s with seg[s].start <= e < seg[s].end.
 * The gc_segments struct is host memory; seg/chunk_seg are device arrays the
 * caller fills once per parameter list (gc_segments_plan builds their host
 * images) and reuses every step.  chunk_seg[c] = the first segment holding
 * element c << chunk_shift, so a kernel finds any element's tensor with two
 * dependent loads (chunk -> record) plus a rare forward walk, no search.
 * Tensors may be empty and have any 4-byte alignment. */
typedef struct gc_seg {
    uint64_t start;    /* first flat element */
    uint64_t end;      /* one past the last */
    float *ptr;        /* device base pointer of the tensor (contiguous fp32) */
    uint64_t reserved; /* 0 (records are 32 bytes) */
} gc_seg;
struct gc_segments {
    uint64_t count;            /* tensors */
    uint64_t n;                /* total elements = seg[count-1].end */
    const gc_seg *seg;         /* device, count records; a sentinel is not needed */
    const uint32_t *chunk_seg; /* device, gc_segments_chunks(n, chunk_shift) entries */
    uint32_t chunk_shift;      /* 4..30 */
    uint32_t sizes_hash;       /* gc_segments_sizes_hash of the tensor sizes, or 0 (unknown) */
};
uint64_t gc_segments_chunks(uint64_t n, uint32_t chunk_shift);
/* a nonzero 32-bit hash of the per-tensor sizes (FNV-1a over the count and each size):
 * calls that pair two tables (gc_segments_copy) refuse two nonzero hashes that differ */
uint32_t gc_segments_sizes_hash(const uint64_t *sizes, uint64_t count);
/* host: (sizes[count], device ptrs[count]) -> seg[count], chunk_seg[chunk_capacity >=
 * gc_segments_chunks(n, chunk_shift)] (host buffers to upload); *n_out = total elements */
int gc_segments_plan(const uint64_t *sizes, float *const *ptrs, uint64_t count, uint32_t chunk_shift,
                     gc_seg *seg, uint32_t *chunk_seg, uint64_t chunk_capacity, uint64_t *n_out);
/* flat[e] = tensor element e (flat may be NULL: max-norm only) and *norm = max |x| over all tensors;
 * workspace as for gc_absmax_f32.  = TensorBuffer(grad_in) + buffer.abs().max() in one pass. */
int gc_segments_flatten_absmax(const gc_segments *segs, float *flat, float *norm, void *workspace,
                               gc_stream_t stream);
/* tensor element e = RN(flat[e] * alpha) + 0.0f — the setgrad loop `out[:] = 0; out.add_(g, alpha)`
 * (reducer.py:543-549, 755-761); the + 0 maps -0 to +0 exactly as the reference does */
int gc_segments_scatter(const float *flat, float alpha, const gc_segments *segs, gc_stream_t stream);
/* dst tensor element e = RN(src tensor element e * alpha) + 0.0f for two lists of the same tensor sizes
 * (the GlobalRandK setgrad of every coordinate, reducer.py:759-761, tensor to tensor).  The host
 * checks the tensor count, the total n and, when both tables carry one, sizes_hash; per-tensor
 * sizes that differ under equal count and n with a zero hash are undefined behaviour (the records
 * live on the device and are not read back) */
int gc_segments_copy(const gc_segments *src, const gc_segments *dst, float alpha, gc_stream_t stream);
/* the GlobalRandK decode-scatter (gc_qsgd_decode with idx) into the tensors of segs:
 * element idx[i] = RN(decode_i * alpha) (reducer.py:754 + 759-761).  Like the
 * flat form, the indices are not range-checked on the device: every idx[i]
 * must be in [0, segs->n) */
int gc_qsgd_decode_scatter_segments(const uint32_t *words, const int64_t *idx, uint64_t k, const float *norm,
                                    uint32_t bits, const gc_lanes *lanes, float alpha, const gc_segments *segs,
                                    gc_stream_t stream);
/* gc_qsgd_decode writing each element straight into its tensor (decode + 1/W + setgrad fused) */
int gc_qsgd_decode_segments(const uint32_t *words, uint64_t n, const float *norm, uint32_t bits,
                            const gc_lanes *lanes, float alpha, const gc_segments *segs, gc_stream_t stream);

/* ---- multi-scale / two-scale --------------------------------------------- */
int gc_ms_mask_encode(const float *x, const int64_t *idx, uint64_t n, const float *norm, const gc_levels *levels,
                      const gc_rng *rng, const gc_lanes *mask_lanes, uint32_t *mask_words, gc_stream_t stream);
/* W = 1 (the MIN over one rank is the identity): gc_ms_mask_encode + gc_ms_select_encode in ONE
 * pass over x, both streams bit-identical to the two-pass encode.  Needs the coupled W = 1 layouts
 * (gc_ms_layout / gc_ms_mask_layout with world = 1), a dense 16-byte aligned x, n < 2^32 and 2 or 3
 * levels of <= 24 bits (GC_EINVAL otherwise: run the two passes). */
int gc_ms_encode_w1(const float *x, uint64_t n, const float *norm, const gc_levels *levels, const gc_rng *rng,
                    const gc_lanes *mask_lanes, const gc_lanes *q_lanes, uint32_t *mask_words, uint32_t *words,
                    gc_stream_t stream);
/* mask_words: the (W-summed) thermometer stream; selected level m = #fields with sum == W */
int gc_ms_select_encode(const float *x, const int64_t *idx, uint64_t n, const float *norm,
                        const gc_levels *levels, const gc_rng *rng, const uint32_t *mask_words,
                        const gc_lanes *mask_lanes, const gc_lanes *q_lanes, uint32_t *words,
                        gc_stream_t stream);
/* q cache — compressors.py:778-797 compress_cache (every level's sign*xi, kept
 * between compress_mask and compress) in packed form: one cell of
 * *bytes_per_element (1 or 2) bytes per element holding every level's select
 * lane.  0 when these levels / n have no cache form (dense wave-split kernels
 * only: 2 or 3 levels of <= 24 bits, n < 2^32, count * bit_length(2 qmax) <= 16). */
int gc_ms_cache_bytes(uint64_t n, const gc_levels *levels, uint32_t *bytes_per_element);
/* gc_ms_mask_encode (dense, 16-byte aligned x) that also writes the cells into
 * cache[n * bytes_per_element] (16-byte aligned) */
int gc_ms_mask_encode_cached(const float *x, uint64_t n, const float *norm, const gc_levels *levels,
                             const gc_rng *rng, const gc_lanes *mask_lanes, uint32_t *mask_words, void *cache,
                             gc_stream_t stream);
/* gc_ms_select_encode from the cells instead of x and the draws: the same words
 * bit for bit for the x / norm / rng the cache was written with */
int gc_ms_select_cached(const void *cache, uint64_t n, const gc_levels *levels, const uint32_t *mask_words,
                        const gc_lanes *mask_lanes, const gc_lanes *q_lanes, uint32_t *words, gc_stream_t stream);
/* order 0: RN(RN(Q*norm)/s_m) (multi-scale); order 1: RN(RN(norm/s_m)*Q) (two-scale); then *alpha */
int gc_ms_decode(const uint32_t *words, const uint32_t *mask_words, const int64_t *idx, uint64_t n,
                 const float *norm, const gc_levels *levels, const gc_lanes *mask_lanes,
                 const gc_lanes *q_lanes, int order, float alpha, float *out, gc_stream_t stream);
/* gc_ms_decode writing each element straight into its tensor */
int gc_ms_decode_segments(const uint32_t *words, const uint32_t *mask_words, uint64_t n, const float *norm,
                          const gc_levels *levels, const gc_lanes *mask_lanes, const gc_lanes *q_lanes, int order,
                          float alpha, const gc_segments *segs, gc_stream_t stream);
/* the GlobalRandK two-scale decode-scatter (gc_ms_decode with idx) into the
 * tensors of segs: element idx[i] = RN(decode_i * alpha) + 0 (reducer.py:1617-1628:
 * decompress, scatter into the flat buffer, setgrad x 1/W).  Every idx[i] must
 * be in [0, segs->n) (not range-checked on the device) */
int gc_ms_decode_scatter_segments(const uint32_t *words, const uint32_t *mask_words, const int64_t *idx, uint64_t k,
                                  const float *norm, const gc_levels *levels, const gc_lanes *mask_lanes,
                                  const gc_lanes *q_lanes, int order, float alpha, const gc_segments *segs,
                                  gc_stream_t stream);
/* unpacked selected level per element (int8), from a thermometer stream */
int gc_ms_mask_unpack(const uint32_t *mask_words, const gc_lanes *mask_lanes, uint32_t levels_count,
                      int8_t *mask, gc_stream_t stream);
/* unpacked forms (the literal compressor drop-ins): int8 resolution mask
 * (compressors.py:799-807), select (809-817), decompress (819-826 / 668-680) */
int gc_ms_quantize_mask(const float *x, uint64_t n, const float *norm, const gc_levels *levels, const gc_rng *rng,
                        int8_t *mask, gc_stream_t stream);
int gc_ms_select_quantize(const float *x, uint64_t n, const float *norm, const gc_levels *levels,
                          const gc_rng *rng, const int8_t *mask, void *q, uint32_t q_dtype, gc_stream_t stream);
int gc_ms_dequantize(const void *q, uint32_t q_dtype, const int8_t *mask, uint64_t n, const float *norm,
                     const gc_levels *levels, int order, float alpha, float *out, gc_stream_t stream);

/* ---- torch CPU generator stream (MT19937) -------------------------------- */
/* state = 624 words + next index (625 uint32); index 624 = block exhausted */
int gc_mt19937_seed(uint64_t seed, uint32_t *state_host);
/* out[count] = next `count` draws; state_dev (625 words, device) advances.
 * One workgroup walks the serial stream (reference / small counts). */
int gc_mt19937_generate(uint32_t *state_dev, uint32_t *out, uint64_t count, gc_stream_t stream);

/* Parallel form of the same stream (bit-identical draws and final state):
 * generator g of G = ceil(count / GC_MT_JUMP_DRAWS) emits draws [g*J, (g+1)*J)
 * from the state jumped g*J draws ahead (GF(2) jump polynomials x^(g*J-1) mod P,
 * P the characteristic polynomial of MT19937).  The jump table depends only on
 * g: gc_mt19937_jump_table fills table_host[count * 624] with the coefficients
 * of generators first .. first+count-1 (first >= 1; host computation, PCLMUL
 * when available); callers upload it once and keep it.  workspace:
 * gc_mt19937_workspace_size(count) device bytes, no initialisation. */
#define GC_MT_JUMP_DRAWS 262080u /* 624 x 420 draws per generator */
int gc_mt19937_jump_table(uint64_t first, uint64_t count, uint32_t *table_host);
size_t gc_mt19937_workspace_size(uint64_t count);
int gc_mt19937_generate_jumped(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint32_t *out,
                               uint64_t count, void *workspace, gc_stream_t stream);
/* the same with generators of J draws (J a positive multiple of 624): the
 * table must then come from gc_mt19937_jump_table_j with the same J, and the
 * workspace is gc_mt19937_workspace_size_j(count, J) bytes.  A J near
 * count / (number of CUs) balances the generator kernel over the chip. */
int gc_mt19937_jump_table_j(uint64_t J, uint64_t first, uint64_t count, uint32_t *table_host);
size_t gc_mt19937_workspace_size_j(uint64_t count, uint64_t J);
int gc_mt19937_generate_jumped_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                 uint32_t *out, uint64_t count, void *workspace, gc_stream_t stream);
/* the same run in two halves: phase 1 = the state's sequence + the jumps (the
 * LDS-bound part), phase 2 = the generators (writes out and advances
 * state_dev), phase 3 = both.  Enqueue 1 then 2 on one stream with identical
 * arguments; an event between them marks the end of the jumps. */
int gc_mt19937_generate_phase_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                uint32_t *out, uint64_t count, void *workspace, int phase, gc_stream_t stream);
/* the run split so that the END STATE is known before any draw exists (for
 * pipelining back-to-back calls): phase 1 = the sequence + the jumps + one more
 * jump to the state after `count` draws, written over state_dev (625 words);
 * phase 2 = the generators (out only; they read the workspace, not state_dev,
 * so the next run's phase 1 may start on another stream once this phase 1 is
 * done, with its own workspace).  end_block = floor((idx + count - 1) / 624)
 * for the state's read index idx (the host knows it: torch's generator state);
 * end_coef = gc_mt19937_jump_table_j(624 * end_block, 1, 1) on the device
 * (NULL when end_block = 0).  The new read index is idx + count - 624 end_block;
 * an end_block that does not match idx yields an index above 624.  Workspace as
 * gc_mt19937_workspace_size_j(count, J). */
int gc_mt19937_generate_split_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                const uint32_t *end_coef, uint64_t end_block, uint32_t *out, uint64_t count,
                                void *workspace, int phase, gc_stream_t stream);
/* One run of nend * per_end draws with nend end states (several same-size
 * calls' draws made by one set of generators: the generator jumps, the
 * LDS-bound part, are shared by the nend calls).  End k = the state after
 * (k + 1) * per_end draws (624 words + read index) goes to
 * ends_out[k * 626 ..]; the last one also over state_dev, so the next run
 * chains from it.  end_coefs (device): nend tables of 624 words, table k =
 * gc_mt19937_jump_table_j(624 * B_k, 1, 1) with B_k = floor((idx + (k + 1) *
 * per_end - 1) / 624), idx = the state's read index (per_end >= 624).
 * workspace: gc_mt19937_workspace_size_multi_j(nend * per_end, J, nend).
 * Phases as gc_mt19937_generate_split_j (1: sequence, jumps, end states; 2:
 * the generators). */
size_t gc_mt19937_workspace_size_multi_j(uint64_t count, uint64_t J, uint32_t nend);
int gc_mt19937_generate_multi_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                const uint32_t *end_coefs, uint32_t nend, uint64_t per_end, uint32_t *ends_out,
                                uint32_t *out, void *workspace, int phase, gc_stream_t stream);
/* gc_mt19937_generate_multi_j with the draws packed to 24 bits (the
 * GC_RNG_STREAM24 layout: 3 per_end / 4 words per call, calls back to back).
 * idx = the state's read index (state_dev[624], which the caller sent); idx
 * and per_end must be multiples of 4, so every call's draws start on a whole
 * word. */
int gc_mt19937_generate_multi24_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                  const uint32_t *end_coefs, uint32_t nend, uint64_t per_end, uint64_t idx,
                                  uint32_t *ends_out, uint32_t *out, void *workspace, int phase, gc_stream_t stream);
/* gc_mt19937_generate_multi_j writing split-plane draws (GC_RNG_SPLIT8 /
 * SPLIT16 for hi_bits 8 / 16): call k's draws form one region of
 * gc_rng_split_bytes(per_end, hi_bits) bytes at out + slot * that, slot = k
 * (ring = 0) or (ring0 + k) % ring (ring >= 2: a ring of regions, ring0 <
 * ring).  Phase 2 runs generators g_first .. g_first + g_count - 1 of the run
 * (g_count = UINT64_MAX: all); generator g's draws [g J, (g + 1) J) may end in
 * the next call's region.  Any read index and per_end (>= 624); out 16-byte
 * aligned.  gc_rng_split_bytes returns 0 for other hi_bits. */
uint64_t gc_rng_split_bytes(uint64_t n, uint32_t hi_bits);
int gc_mt19937_generate_multi_split_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                      const uint32_t *end_coefs, uint32_t nend, uint64_t per_end, uint64_t idx,
                                      uint32_t hi_bits, uint32_t *ends_out, void *out, uint32_t ring, uint32_t ring0,
                                      uint64_t g_first, uint64_t g_count, void *workspace, int phase,
                                      gc_stream_t stream);
/* gc_mt19937_generate_split_j with the draws packed to 24 bits (the
 * GC_RNG_STREAM24 layout: 3 count / 4 words of out).  idx = the state's read
 * index (state_dev[624], which the caller sent); idx and count must be
 * multiples of 4, so every 4 draws fill 3 whole words. */
int gc_mt19937_generate_split24_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                  const uint32_t *end_coef, uint64_t end_block, uint32_t *out, uint64_t count,
                                  uint64_t idx, void *workspace, int phase, gc_stream_t stream);
/* torch-mode QSGD quantize with the MT19937 draws consumed in-kernel (never
 * stored): q[i] = sign(x_i)*xi_i exactly as compressors.py:299-316 computes it
 * under torch.bernoulli (one draw per element, in order), as GC_I8 (bits <= 7)
 * or GC_I32 (the reference's _dtype, compressors.py:294-297).  state_dev
 * advances by n draws, like gc_mt19937_generate_jumped_j with the same J,
 * table and workspace (gc_mt19937_workspace_size_j(n, J)).  Pack with
 * gc_lane_pack. */
int gc_qsgd_quantize_mt19937(const float *x, uint64_t n, const float *norm, uint32_t bits, uint32_t *state_dev,
                             const uint32_t *table_dev, uint64_t table_gens, uint64_t J, void *q, uint32_t q_dtype,
                             void *workspace, gc_stream_t stream);

/* ---- reference-compatible packers ----------------------------------------- */
/* greedy 4-mode format of extensions/Extension CPU/bitpacking.cpp (host
 * buffers); returns words / elements written or a negative status */
int64_t gc_greedy4_pack(const int32_t *src, uint64_t n, int32_t *out, uint64_t cap);
int64_t gc_greedy4_unpack(const int32_t *src, uint64_t nwords, int32_t *out, uint64_t cap);
/* 8 x (v & 0xFF) per int64, MSB-first (extensions/Extension CPU BP), device */
int gc_bytepack8(const void *src, uint32_t src_dtype, uint64_t n, int64_t *out, gc_stream_t stream);
int gc_byteunpack8(const int64_t *src, uint64_t nwords, int8_t *out, gc_stream_t stream);
/* QSGDBPCompressor.decompress (compressors.py:375-376) after the two greedy4
 * unpacks: out[i] = (*c * (sign[i] == 1 ? -1 : 1)) * (float)xi[i], device
 * buffers, 16-byte aligned (c = RN(norm / s) as compress returns it) */
int gc_qsgdbp_decode(const int32_t *sign, const int32_t *xi, uint64_t n, const float *c, float *out,
                     gc_stream_t stream);
/* host-buffer forms (the reference's byte packer is a CPU extension) */
int gc_bytepack8_host(const int64_t *src, uint64_t n, int64_t *out);
int gc_byteunpack8_host(const int64_t *src, uint64_t nwords, int8_t *out);

#ifdef __cplusplus
}
#endif
#endif /* GCODEC_H */
