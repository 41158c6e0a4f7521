/*
 * replicat_chunker.h -- C ABI of the MI355X (gfx950) content-defined chunker.
 *
 * Drop-in boundary for replicat's native chunker module `_replicat_adapters`
 * (/root/reference/src/adapters.cpp:80-86, stub stubs/_replicat_adapters.pyi:3-8).
 * Plain pointers and sizes only; no torch types.  Implemented by
 * replicat_amd/csrc/{capi.cpp,kernels.hip} -> replicat_amd/libreplicat_chunker.so.
 *
 * The chunk rule reproduced bit for bit:
 *   key(p)   = k1 ^ lo(k0 (x) d) ^ lo(0x1B (x) hi(k0 (x) d)),  d = LE64(buf[p-4 .. p+4])
 *              (x) = carry-less multiply          -- adapters.cpp:72-77
 *   next_cut = first argmax of key over p = 4, 8, .. < max_length, forced up to
 *              roundup4(min_length); tail rules for a final buffer < 2*max_length
 *                                                  -- adapters.cpp:42-70
 *   framing  = a stream of L bytes whose last piece starts at byte P is chunked exactly as
 *              replicat's Python adapter loop chunks its pieces  -- adapters.py:290-305
 *
 * Error codes: RC_OK, or one of the reference constructor's three ValueErrors
 * (adapters.cpp:21-29, same check order), or an RC_ERR_* of this library.
 * rc_last_error() returns the message of the calling thread's last failure.
 */
#ifndef REPLICAT_CHUNKER_H
#define REPLICAT_CHUNKER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RC_OK 0
#define RC_ERR_KEY_LENGTH 1 /* "key must contain exactly 16 characters"          adapters.cpp:21-22 */
#define RC_ERR_MIN_GT_MAX 2 /* "Minimum length is greater than the maximum one"  adapters.cpp:23-24 */
#define RC_ERR_BAD_KEY 3    /* "Bad key contents" (k0 == 0)                      adapters.cpp:28-29 */
#define RC_ERR_ARGUMENT 10  /* bad pointer / size / P > L                                       */
#define RC_ERR_ALIGN 11     /* a device stream base is not 16-byte aligned                      */
#define RC_ERR_HIP 12       /* a HIP runtime call failed (message in rc_last_error)             */
#define RC_ERR_OVERFLOW 13  /* a stream produced more cuts than its capacity (never expected)   */
#define RC_ERR_NO_DEVICE 14 /* no usable gfx950 device                                          */
#define RC_ERR_DEVICE_FAULT 15 /* the tile kernel took its fail-safe stop (a workgroup grab never
                              published, kernels.hip UnitGrab): that call's cuts are not the
                              reference's and were not returned (never observed)               */

/* Per-stream counts written by rc_chunk_device besides the cut count itself */
#define RC_COUNT_OVERFLOW (-1) /* the stream produced more cuts than its capacity (never expected) */
#define RC_COUNT_FAULT (-3)    /* the call's tile kernel took its fail-safe stop: EVERY stream of
                                  the call gets this count and none of its cuts is valid
                                  (RC_ERR_DEVICE_FAULT on the blocking paths)                    */

/* rc_chunk_* flags */
#define RC_OPEN 1u /* every stream is an OPEN prefix: its bytes all belong to non-final pieces, so
                      the chain cuts only while L - s >= max_length and never applies the tail
                      rule (the adapter's non-final next_cut calls, adapters.py:295-301); the
                      uncut remainder starts at the last reported cut (0 if none).  last_piece is
                      ignored. */
#define RC_PIPELINED 2u /* (rc_chunk_device) run the call on the chunker's two CU-partitioned
                      streams (rc_chunker_overlap): the tile kernel on most CUs, the edge and
                      chain kernels on the reserved ones, so that this call's chain runs beside
                      the NEXT call's tile kernel.  The tile kernel waits for the work queued on
                      hip_stream before the call (the inputs); hip_stream does not wait for the
                      outputs -- rc_chunk_wait does.  Same cuts as without the flag.  The
                      chunker's streams are blocking streams (HIP creates CU-masked streams so):
                      a caller on the legacy NULL stream gets correct but serial calls, so
                      pipelined callers use a non-blocking stream.  Calls the overlap does not
                      pay for run in sequence on hip_stream instead (a legal schedule of the
                      flag): chunkers with small windows (max_length below ~1 MB: the chain
                      does not fit beside the tile kernel) and batches with fewer 16 KiB
                      tiles of needed bytes than the masked tile kernel has waves (~56 MiB on
                      224 CUs; e.g. short streams whose keys are never needed: nothing to
                      overlap the chain with).
                      RC_PIPE_ALL=1 in the environment pipelines every call.  The streams'
                      bytes and the outputs must stay allocated until the call is waited for:
                      a caching allocator (torch's) sees only the caller's stream, which a
                      pipelined call's kernels do not run on. */
#define RC_PIPELINE_END 4u /* (with RC_PIPELINED) the last call of a sequence: no tile kernel
                      follows for its chain to run beside, so its edge and chain kernels run on
                      every CU (config 2: ~0.2 ms instead of ~0.75 ms on the reserved CUs). */

typedef struct rc_chunker rc_chunker;

/* Library / ABI version: 300 = 0.3.0 (replicat_amd.__version__; tests/test_cabi.py checks they agree). */
int rc_version(void);

/* Build id: a hash over the library's sources and compile flags, set by replicat_amd/build.py
 * ("unknown" for a build outside it).  Profiles record it so stale counters are refused. */
const char *rc_build_id(void);

/* Message of this thread's last error ("" if none). */
const char *rc_last_error(void);

/* Constructor of `_gclmulchunker(min_length, max_length, key)` (adapters.cpp:18-34):
 * validates key_len == 16, min <= max, k0 != 0 in that order, then builds the GF(2) lookup
 * tables of the key and uploads them to `device` (a HIP device ordinal).  On success *out owns
 * device memory until rc_chunker_destroy. */
int rc_chunker_create(uint64_t min_length, uint64_t max_length, const uint8_t *key,
                      uint64_t key_len, int device, rc_chunker **out);
void rc_chunker_destroy(rc_chunker *ch);

/* The readonly `min_length` / `max_length` attributes (adapters.cpp:83-84). */
uint64_t rc_chunker_min_length(const rc_chunker *ch);
uint64_t rc_chunker_max_length(const rc_chunker *ch);

/* `next_cut(buffer, final)` (adapters.cpp:42-70) on a HOST buffer: returns the cut length
 * in *out_cut (0 = "need more data").  Tail and wait decisions are taken on the host; an
 * argmax copies the first <= max_length+3 bytes to the device, runs the device kernels and
 * waits for the answer.  Blocking. */
int rc_next_cut(rc_chunker *ch, const uint8_t *buffer, uint64_t size, int final,
                uint64_t *out_cut);

/* Capacity (in cuts) that stream i of length lens[i] needs: caps[i] = L / max(4, roundup4(min))
 * + 3.  Returns the sum over all n streams (the size of the `cuts` array below). */
uint64_t rc_cut_capacity(const rc_chunker *ch, uint64_t n, const uint64_t *lens,
                         uint64_t *caps /* may be NULL */);

/* Batch entry point over DEVICE-resident streams (the batching shim of SURVEY.md §8 b):
 *   d_streams[i]  device pointer to stream i (16-byte aligned), lens[i] = L_i bytes,
 *   last_piece[i] = P_i, start of the stream's last piece (0 = one piece; P_i <= L_i).
 * Writes stream i's chunk END offsets (u64, relative to the stream) to
 * d_cuts[cut_base[i] ..] where cut_base = exclusive prefix sum of the capacities of
 * rc_cut_capacity, and the count to d_counts[i] (int64; RC_COUNT_OVERFLOW = capacity overflow,
 * RC_COUNT_FAULT = the call's tile kernel took its fail-safe stop -- every count of the call is
 * then RC_COUNT_FAULT: a caller that reads the counts must treat any negative one as an error).
 * The host arrays are read before return; the work is enqueued on `hip_stream` (a
 * hipStream_t, NULL = default stream) and the call returns without synchronising.  With
 * RC_PIPELINED the kernels go to the chunker's own streams instead (see the flag). */
int rc_chunk_device(rc_chunker *ch, uint64_t n, const uint8_t *const *d_streams,
                    const uint64_t *lens, const uint64_t *last_piece, uint32_t flags,
                    uint64_t *d_cuts, int64_t *d_counts, void *hip_stream);

/* Overlap mode of RC_PIPELINED calls: keep `reserve_cus` CUs (0 = the default, 32, or
 * RC_OVERLAP_CUS) for the edge and chain kernels and give the tile kernel the rest.  The split
 * is a pair of CU-masked HIP streams (hipExtStreamCreateWithCUMask; a multiple of 32 reserves
 * the same number of CUs on every shader engine of every XCD -- anything else leaves engines
 * unequal, and the persistent tile kernel slows by ~15 %); changing it waits for the pipelined
 * calls in flight.
 * rc_chunker_overlap_cus returns the current split (0 before the first pipelined call). */
int rc_chunker_overlap(rc_chunker *ch, uint32_t reserve_cus);
uint32_t rc_chunker_overlap_cus(const rc_chunker *ch);
/* How many RC_PIPELINED calls so far ran on the two streams (the rest ran in sequence). */
uint64_t rc_chunker_pipelined_calls(const rc_chunker *ch);

/* Make hip_stream wait (device side, no host synchronisation) until every rc_chunk_device call
 * made so far -- pipelined or not -- has written its cuts and counts. */
int rc_chunk_wait(rc_chunker *ch, void *hip_stream);

/* A HIP stream on `device` with a hardware queue of its own (no reference counterpart:
 * plumbing for device-side overlap).  Plain HIP streams share the process's GPU_MAX_HW_QUEUES
 * hardware queues (4 by default) and a kernel queued behind another stream's long kernel on the
 * same queue waits for it; a stream created with a CU mask never shares its queue, so this one is
 * created with every CU in its mask (hipExtStreamCreateWithCUMask).  Like every CU-masked stream
 * it is a BLOCKING stream: work on the legacy NULL stream synchronises with it.  The snapshot
 * producer's batch streams use it so that consecutive batches' digests (each ending with a
 * ~55 ms BLAKE2b chain) overlap at HIP's default queue count.  rc_stream_destroy waits for the
 * stream's work; streams still alive at process exit are destroyed then (the library's exit
 * hook).  Do NOT destroy a stream another runtime has wrapped and may still record events on
 * (torch's caching allocator records one on every stream a freed tensor was used on, possibly
 * long after): leave it to the exit hook -- replicat_amd.chunker.QueueStream.close() retires
 * such a stream instead of destroying it.  Each stream holds one hardware queue of its own. */
int rc_stream_create(int device, void **out_stream);
void rc_stream_destroy(void *stream);

/* The same over HOST-resident streams, blocking: pinned double-buffered H2D copies overlap
 * the kernels of the previous batch; cuts come back to host arrays laid out as above
 * (cuts[cut_base[i] ..], counts[i]).  This is the end-to-end path of DESIGN.md. */
int rc_chunk_host(rc_chunker *ch, uint64_t n, const uint8_t *const *streams,
                  const uint64_t *lens, const uint64_t *last_piece, uint32_t flags,
                  uint64_t *cuts, int64_t *counts);

/* Waits for the chunker's calls so far and reports tile-kernel fail-safe stops: with
 * workgroup grabs (RC_TILE_GROUP) a wave that waited ~1 s for its group's grab to be published
 * stops rather than hang the GPU, leaving that launch's records incomplete (its counts are then
 * RC_COUNT_FAULT, and rc_next_cut / rc_chunk_host fail with RC_ERR_DEVICE_FAULT).  RC_OK, or
 * RC_ERR_DEVICE_FAULT with rc_last_error() giving how many calls faulted since the previous
 * check; the count restarts at every check.  (Never observed outside the diagnostic build that
 * forces it, diag/lib_GRABFAULT.so.)  Not a reference interface: replicat has no device. */
int rc_chunker_check(rc_chunker *ch);

/* Kernel timing, for bench.py's roofline: while enabled, every rc_chunk_device call records
 * HIP events on the launch stream before the tile kernel, between it and the edge kernel, and
 * around the chain kernels.  rc_timing_read_kernels waits for the recorded events, returns the
 * summed milliseconds of each phase and the number of calls, and clears the record;
 * rc_timing_read returns phase A = tile + edge and phase B = chain the same way. */
int rc_timing_enable(rc_chunker *ch, int enable);
int rc_timing_read_kernels(rc_chunker *ch, double *tile_ms, double *edge_ms, double *chain_ms,
                           uint64_t *calls);
int rc_timing_read(rc_chunker *ch, double *phase_a_ms, double *phase_b_ms, uint64_t *calls);

/* Synthetic stream bytes on the device (replicat_amd/synth.py): word i of stream `stream`
 * is splitmix64((seed * 0x9E3779B97F4A7C15) ^ (stream << 34) ^ i), little-endian. */
int rc_fill_splitmix(uint8_t *d_dst, uint64_t nbytes, uint64_t seed, uint64_t stream,
                     void *hip_stream);
/* n streams at once, stream k (id first_stream + k * stream_step) at d_dst + k * slot; slot
 * is a multiple of 8 of at least nbytes rounded up to 8 (a stream's last word is written whole,
 * into the slot's slack).  One launch for a whole arena of synthetic streams. */
int rc_fill_splitmix_streams(uint8_t *d_dst, uint64_t n, uint64_t nbytes, uint64_t slot,
                             uint64_t seed, uint64_t first_stream, uint64_t stream_step,
                             void *hip_stream);
/* The same bytes from word `word0` of the stream on (byte offset 8 * word0): one segment of a
 * long stream (the multi-device split of a single stream, replicat_amd/split.py). */
int rc_fill_splitmix_at(uint8_t *d_dst, uint64_t nbytes, uint64_t seed, uint64_t stream,
                        uint64_t word0, void *hip_stream);

/* Calibration (bench.py --calibrate): stream the first nbytes (whole 16 KiB tiles) of a
 * 16-byte aligned device buffer with the tile kernel's exact load pattern and work schedule
 * (static ranges + grabbed units) and no hashing; its rate is the attainable streaming-read
 * ceiling for the tile kernel on this device.  d_out: 4 u32 of device scratch (d_out[1] is the
 * schedule's grab counter, zeroed by the call on its stream).  Enqueue only. */
int rc_read_probe(const uint8_t *d_src, uint64_t nbytes, uint32_t *d_out, void *hip_stream);
/* The same probe under one chunker's tile schedule (the RC_TILE_* knobs it was created with),
 * so that schedules can be compared in one process on one allocation (scripts/). */
int rc_chunker_read_probe(rc_chunker *ch, const uint8_t *d_src, uint64_t nbytes, uint32_t *d_out,
                          void *hip_stream);

/* Keys j (key j covers bytes [4j-4, 4j+4)) that any argmax window of a stream (L, P) can
 * reach: the largest such j, or 0 when the stream never hashes (tail rule only). */
uint64_t rc_keys_needed(uint64_t max_length, uint64_t L, uint64_t P);

/* One 64-bit key of the chunker on the host, from its lookup tables (tests / tooling). */
uint64_t rc_host_key(const rc_chunker *ch, uint64_t d);

/* Inspection (tests): run only the per-tile phase (tile + edge kernels) over device streams and
 * copy the tile records to host arrays: for tile t of the concatenated tile list (stream i's
 * tiles start at the exclusive prefix sum of jneed_i / rc_tile_keys() + 1), keys[t] = the first
 * maximal 64-bit key among the tile's keys (0 if none is positive) and js[t] = its key index in
 * the stream.  A tile's keys are all of j0 .. j0 + rc_tile_keys() - 1 when their bytes lie in
 * the stream, else those up to jneed; key 0 never counts.  gmax (may be NULL): for chunkers
 * with small windows (max_length below ~1 MB) the top-16 maximum of each quarter of the tile
 * (u16 q at bits 16q), ~0 for a tile computed exactly or a chunker without them.  ghot (may be
 * NULL, 4 words per tile): ghot[4t + q] bit l = lane l of the tile kernel (which holds keys
 * 256 i + 4 l .. 256 i + 4 l + 3 of each of the quarter's iterations i) has a key in quarter q
 * whose top 16 bits reach rc_group_hot_threshold(ch); all ones where gmax is ~0.  *n_tiles
 * receives the tile count; at most cap are copied.  Blocking. */
int rc_tile_records(rc_chunker *ch, uint64_t n, const uint8_t *const *d_streams,
                    const uint64_t *lens, const uint64_t *last_piece, uint64_t *keys,
                    uint64_t *js, uint64_t *gmax, uint64_t *ghot, uint64_t cap,
                    uint64_t *n_tiles);
/* The top-16 value from which a lane of a tile quarter counts as hot in rc_tile_records (a
 * function of max_length: 10 / window of the 16-bit range below the top; 0 = none). */
uint32_t rc_group_hot_threshold(const rc_chunker *ch);
uint64_t rc_tile_keys(void);

/* Host-only inspection of the tile kernel's work units (tests; no device needed): the units a
 * launch over n_tiles tiles by `waves` waves hands out under the schedule knobs (RC_TILE_STATIC,
 * RC_TILE_CHUNK, RC_TILE_DYN_MIN): unit u covers tiles [ranges[2u], ranges[2u + 1]); *n_units
 * receives the count, at most cap are written. */
int rc_tile_schedule(uint64_t n_tiles, uint32_t waves, uint32_t permille, uint32_t chunk,
                     uint32_t dyn_min, uint32_t *ranges, uint64_t cap, uint64_t *n_units);

/* Host-only check of the table construction (no device needed): out[i] = key of data word
 * ds[i] under the 16-byte key, evaluated from the same byte tables the kernels use, and
 * top16[i] = its top 16 bits as the prefilter tables give them. */
int rc_tables_key(const uint8_t *key16, uint64_t n, const uint64_t *ds, uint64_t *out,
                  uint32_t *top16);

#ifdef __cplusplus
}
#endif

#endif /* REPLICAT_CHUNKER_H */
