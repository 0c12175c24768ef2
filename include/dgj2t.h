/*
 * dgj2t.h — C ABI of the MI355X-native batched JSON -> Thrift-binary
 * transcoder (the conv/j2t hot path of cloudwego/dynamicgo).
 *
 * Boundary replaced (reference, Go -> machine code, no cgo):
 *   J2T_FSM(fsm *types.J2TStateMachine, buf *[]byte, src *string, flag uint64) uint64
 *     internal/native/dispatch_amd64.go:66-68
 *   -> uint64_t j2t_fsm_exec(J2TStateMachine*, GoSlice *buf, const GoString *src, uint64_t flag)
 *     native/thrift.h:202, native/thrift.c:765-1187
 * and the Go prelude/epilogue around it (BinaryConv.do conv/j2t/impl.go:38-91,
 * BinaryConv.Do conv/j2t/conv.go:53-77).
 *
 * The reference converts ONE message per call, reading Go descriptor structs
 * in place. This ABI converts a BATCH: a JSON arena with n+1 offsets, against a
 * descriptor flattened once (include/dgj2t_desc.h) and kept resident on the
 * device. Per message it returns the Thrift bytes and the reference's packed
 * status word, bit-identical: code bits 0-7 | pos bits 8-39 | value bits 40-63
 * (native/thrift.h:223-242, decoded by explainNativeError
 * conv/j2t/impl_amd64.go:261-298), 0 = success.
 *
 * Flags are the reference's j2t flag word (native/thrift.h:23-32,
 * conv/j2t/conv.go:98-127 toFlags). DG_F_VALIDATE_UTF8 is an opt-in extension
 * (bit 16) that the reference does not have; off by default. With it, the raw
 * JSON bytes of every string written as a Thrift STRING (string values and
 * STRING map keys; not binary fields, not field-name keys) must be valid UTF-8
 * as utf8_validate (native/utf8.c:101-212) defines it; otherwise the message
 * fails with ERR_INVAL (2), value = the first byte of the invalid sequence,
 * pos = its offset.
 *
 * All functions return 0 on success and a negative DG_E_* on API failure;
 * dg_last_error() describes the last failure of the calling thread.
 */
#ifndef DGJ2T_H
#define DGJ2T_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#include "dgj2t_defs.h"

typedef struct dg_ctx dg_ctx;
typedef struct dg_desc dg_desc;
typedef struct dg_agg dg_agg;

/* Per-thread description of the last failure. */
const char *dg_last_error(void);

/* "dgj2t-build:<source sha256/16> arch:gfx950": what this library was built
 * from (dynamicgo_amd/build.py); no reference counterpart. */
const char *dg_build_info(void);

/* A context owns one HIP device, a stream and device workspaces. */
int dg_ctx_create(int device, dg_ctx **out);
void dg_ctx_destroy(dg_ctx *ctx);
/* The context's HIP stream (hipStream_t), for callers that order their own work. */
void *dg_ctx_stream(dg_ctx *ctx);
/* Diagnostics (no reference counterpart): messages the kernel's fast path
 * handed to the exact machine, and messages redone with the 4096-deep stack,
 * summed over this context's launches since the last reset. Synchronizes the
 * device. */
int dg_ctx_stats(dg_ctx *ctx, uint64_t *bails, uint64_t *deeps, int reset);

/* Diagnostics: the context's n (<= 16) raw device counters: [0] bails, [1]
 * deep redos, [2..11] wave-kernel phase cycles in a -DDG_WPROF build. */
int dg_ctx_counters(dg_ctx *ctx, uint64_t *out, int n, int reset);

/* Routing knobs (no reference counterpart; testing and tuning). They are read
 * from the environment ONCE, by dg_ctx_create, and changed only through these
 * calls, so routing never changes under a running launch:
 *   "flat"        DG_FLAT         -1 auto, 0 never, 1 always the flat kernel for flat roots
 *   "wave_min"    DG_WAVE_MIN     messages longer than this go to the wave kernel (512)
 *   "wave_occ"    DG_WAVE_OCC     0 auto, 4 or 5: the wave kernel's waves/SIMD instance
 *   "small_mpw"   DG_SMALL_MPW    small-kernel messages per wave (64); 0 = lane kernel
 *   "list_blocks" DG_LIST_BLOCKS  grid of the exact-machine list pass (16)
 *   "t2j_spread"  DG_T2J_SPREAD   0 auto, 1, 2 or 4 lanes per t2j message
 *   "t2j_wave_min" DG_T2J_WAVE_MIN t2j messages longer than this take the t2j wave kernel (512; 0 never)
 *   "flat_wrap"   DG_FLAT_WRAP    -1 auto, 0 off: the flat kernel for {"key":{flat}} members of a non-flat root
 * Unknown names return DG_E_INVALID. Thread-safe (the context lock). */
int dg_ctx_set_knob(dg_ctx *ctx, const char *name, int64_t value);
int dg_ctx_get_knob(dg_ctx *ctx, const char *name, int64_t *value);

/* Upload a dg_desc blob (v1 or v2) (include/dgj2t_desc.h) to the context's device.
 * Replaces reading the Go *thrift.TypeDescriptor graph in place
 * (native/thrift.h:70-137 <-> thrift/descriptor.go:119-267). */
int dg_desc_create(dg_ctx *ctx, const void *blob, size_t len, dg_desc **out);
/* Same, for a blob already resident in device memory (e.g. received by an
 * RCCL broadcast on a non-root rank). */
int dg_desc_create_device(dg_ctx *ctx, const void *d_blob, size_t len, dg_desc **out);
void dg_desc_destroy(dg_desc *desc);
/* Root type index recorded in the blob header. */
uint32_t dg_desc_root(const dg_desc *desc);

/*
 * Device-resident batch: every pointer is device memory of ctx's device.
 *   d_json      JSON arena (at least in_off[n] + 16 readable bytes)
 *   d_in_off    n+1 u64 offsets into d_json; message i = [in_off[i], in_off[i+1])
 *   d_out       output arena; message i may use [out_off[i], out_off[i+1])
 *   d_out_off   n+1 u64 slot bounds (e.g. prefix sum of dg_slot_bound(len))
 *   d_out_len   n u32: Thrift bytes written for message i (0 on error; for
 *               DG_ST_OUT_OVERFLOW: the bytes the message needs)
 *   d_ret       n u64: packed reference status (0 = ok), or DG_ST_OUT_OVERFLOW
 *   d_pending   optional u32 counter (device), incremented once per message
 *               left with DG_ST_OUT_OVERFLOW; may be NULL
 * Enqueued on ctx's stream (or `stream` if non-NULL); asynchronous. ctx's
 * stream is a blocking stream, so it is ordered with the legacy default
 * stream (handle 0) both ways. Launches
 * on different streams of one context may run concurrently: each stream gets
 * its own device scratch (lists, counters, workspaces), up to 40 streams per
 * context (an aggregator's ring of up to 24, the in-flight and pipeline
 * streams); beyond that a shared scratch orders the launches with events, so
 * launches on streams that share one run one after the other.
 * Equivalent, per message, to BinaryConv.Do(ctx, desc, jbytes)
 * (conv/j2t/conv.go:53-77) with the given flags.
 */
int dg_j2t_batch_device(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *d_json,
                        const uint64_t *d_in_off, uint64_t n, uint64_t flags, uint8_t *d_out,
                        const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret,
                        uint32_t *d_pending, void *stream);

/* The same with the batch's longest message length (0 = unknown). The host
 * that built the arena knows it for free; with it the library schedules only
 * the kernels the batch needs (all messages short: the lane kernel alone,
 * no wave-kernel / exact-list launches). */
int dg_j2t_batch_device_ml(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *d_json,
                           const uint64_t *d_in_off, uint64_t n, uint64_t flags, uint8_t *d_out,
                           const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret,
                           uint32_t *d_pending, void *stream, uint64_t max_len);

/* dg_j2t_batch_device_ml for DG_F_HM_SPLIT batches (HTTPConv with the host
 * half of the reference's HTTP-mapping callbacks): d_hm_tab holds n_hm
 * dg_hm_entry per message (dgj2t_defs.h), the bytes handleHttpMappings
 * (conv/j2t/impl.go:243-292) wrote for each struct with mapped fields and the
 * mask of the fields it wrote, into d_hm_bytes. Where the reference returns
 * ERR_HM to Go, the kernel writes the entry's bytes and resumes. A ROOT whose
 * unset fields go to the reference's field cache (F_TRACE_BACK) comes back as
 * DG_ST_HM_END for the host to finish; DG_ST_HM_ERR = the host's entry was an
 * error. d_hm_tab NULL = the root's mapped fields only, all written by the
 * host (its bytes put in front by the caller). */
int dg_j2t_batch_device_hm(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *d_json,
                           const uint64_t *d_in_off, uint64_t n, uint64_t flags, const dg_hm_entry *d_hm_tab,
                           uint32_t n_hm, const uint8_t *d_hm_bytes, uint8_t *d_out, const uint64_t *d_out_off,
                           uint32_t *d_out_len, uint64_t *d_ret, uint32_t *d_pending, void *stream,
                           uint64_t max_len);

/* dg_j2t_batch_device_ml with the host's answers to the reference's Go
 * callbacks (dg_cb_tables, dgj2t_defs.h; device pointers): the HTTP-mapping
 * table of dg_j2t_batch_device_hm and the value-mapping answers (ERR_VM_END,
 * handleValueMapping conv/j2t/impl_amd64.go:117-155). cb NULL = none. */
int dg_j2t_batch_device_cb(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *d_json,
                           const uint64_t *d_in_off, uint64_t n, uint64_t flags, const dg_cb_tables *cb,
                           uint8_t *d_out, const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret,
                           uint32_t *d_pending, void *stream, uint64_t max_len);

/* dg_j2t_batch_device_ml enqueued `iters` times back to back in one call
 * (one lock, no host round trip between batches): a host that re-runs the
 * same job -- benchmarks, replays -- keeps the GPU fed. Every iteration is a
 * complete conversion of the batch. */
int dg_j2t_batch_device_iters(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *d_json,
                              const uint64_t *d_in_off, uint64_t n, uint64_t flags, uint8_t *d_out,
                              const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret,
                              uint32_t *d_pending, void *stream, uint64_t max_len, int iters);

/* dg_j2t_batch_device_iters with HIP timing events around each of the batch's
 * launches (measurement only: the events add a few microseconds between
 * kernels). ms[0] = the first kernel (flat, small or lane), ms[1] = the wave
 * kernel, ms[2] = the list pass (exact machine), each averaged over `iters`
 * serial conversions; 0 for a launch the route does not make. Returns after
 * the stream has drained. */
int dg_j2t_batch_device_ktime(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *d_json,
                              const uint64_t *d_in_off, uint64_t n, uint64_t flags, uint8_t *d_out,
                              const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret,
                              uint32_t *d_pending, void *stream, uint64_t max_len, int iters, double *ms);

/* One in-flight batch's outputs (dg_j2t_batch_device_inflight). */
typedef struct dg_out_set {
    uint8_t *d_out;      /* slot arena, laid out by the shared d_out_off */
    uint32_t *d_out_len;
    uint64_t *d_ret;
    uint32_t *d_pending;
} dg_out_set;

/* `iters` complete conversions of the batch with up to `depth` (1..8) of them
 * in flight at once: conversion k writes sets[k % depth] on the context's
 * k % depth-th stream (stream 0 = `stream`; the others are the context's own,
 * forked from `stream` at the call and joined back into it before return, so
 * work enqueued on `stream` afterwards sees every conversion done). Batch k+1's
 * kernels fill the CUs batch k's tail and list pass leave idle -- what a
 * gateway with several batches from its aggregator in flight runs. depth 1 is
 * dg_j2t_batch_device_iters. */
int dg_j2t_batch_device_inflight(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *d_json,
                                 const uint64_t *d_in_off, uint64_t n, uint64_t flags, const uint64_t *d_out_off,
                                 const dg_out_set *sets, int depth, void *stream, uint64_t max_len, int iters);

/* Output-slot size the device path uses by default for a message of len
 * bytes: 4 len + 64 rounded up to 128 (slots on L2-line boundaries: a line
 * written in part is written back whole). */
uint64_t dg_slot_bound(uint64_t len);

/*
 * Host batch (pinned or pageable host memory): H2D, kernels, overflow reruns,
 * D2H with the outputs compacted. On return out holds the n outputs back to
 * back: message i is out[out_off[i], out_off[i+1]) (empty on error, see ret).
 * out_cap must be >= the total; *out_need receives the total required (if the
 * call returns DG_E_NOMEM because out_cap was too small, retry with it).
 */
int dg_j2t_batch_host(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *json,
                      const uint64_t *in_off, uint64_t n, uint64_t flags, uint8_t *out, uint64_t out_cap,
                      uint64_t *out_off, uint64_t *ret, uint64_t *out_need);

/* dg_j2t_batch_host with the HTTP-mapping table of dg_j2t_batch_device_hm
 * (host memory; hm_bytes of hm_len bytes). DG_ST_HM_END messages keep their
 * partial output (and requires words) in out. */
int dg_j2t_batch_host_hm(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *json,
                         const uint64_t *in_off, uint64_t n, uint64_t flags, const dg_hm_entry *hm_tab, uint32_t n_hm,
                         const uint8_t *hm_bytes, uint64_t hm_len, uint8_t *out, uint64_t out_cap, uint64_t *out_off,
                         uint64_t *ret, uint64_t *out_need);

/* dg_j2t_batch_host with the host's callback answers (dg_cb_tables, host
 * memory): DG_ST_HM_END messages keep their partial output (and requires
 * words) in out, ERR_VM_END messages (code 24) their 16-byte record. */
int dg_j2t_batch_host_cb(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *json,
                         const uint64_t *in_off, uint64_t n, uint64_t flags, const dg_cb_tables *cb, uint8_t *out,
                         uint64_t out_cap, uint64_t *out_off, uint64_t *ret, uint64_t *out_need);

/* One message, BinaryConv.Do semantics (conv/j2t/conv.go:53-77). *out_len is
 * the Thrift length; returns the packed status word through *ret. */
int dg_j2t_do(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *json, size_t len,
              uint64_t flags, uint8_t *out, size_t out_cap, size_t *out_len, uint64_t *ret);

/* Pack the converted messages for the device->host copy: message i's
 * d_out_len[i] bytes move from its slot (d_out + d_out_off[i]) to
 * d_dst + d_dst_off[i], where d_dst_off is the exclusive prefix sum of
 * d_out_len (caller-computed, e.g. one scan kernel). Stream-ordered; errored
 * messages have out_len 0. The Go side then hands (dst, dst_off) to the NIC
 * path without per-message copies. */
int dg_pack_device(dg_ctx *ctx, const uint8_t *d_out, const uint64_t *d_out_off, const uint32_t *d_out_len, uint64_t n,
                   uint8_t *d_dst, const uint64_t *d_dst_off, void *stream);

/* dg_pack_device with the prefix sum folded in (one launch): computes
 * d_dst_off[0..n] = exclusive prefix sum of d_out_len (d_dst_off[n] = total
 * bytes) and packs message i's bytes at d_dst + d_dst_off[i]. Stream-ordered
 * after the conversion that wrote d_out_len. */
int dg_pack_device_scan(dg_ctx *ctx, const uint8_t *d_out, const uint64_t *d_out_off, const uint32_t *d_out_len,
                        uint64_t n, uint8_t *d_dst, uint64_t *d_dst_off, void *stream);

/* HTTPConv framing (conv/j2t/http_conv.go:68-114) fused into the packing:
 * every message that converted (d_ret[i] == 0) is packed as
 * hdr + body + ftr, every failed one as nothing; d_dst_off as in
 * dg_pack_device_scan. hdr/ftr are host bytes (the message header and footer
 * of thrift.GetBinaryMessageHeaderAndFooter, thrift/binary.go:137-175),
 * copied by the call; (hdr_len rounded up to 8) + ftr_len must be <= 4080. */
int dg_pack_device_framed(dg_ctx *ctx, const uint8_t *d_out, const uint64_t *d_out_off, const uint32_t *d_out_len,
                          const uint64_t *d_ret, uint64_t n, const uint8_t *hdr, uint32_t hdr_len, const uint8_t *ftr,
                          uint32_t ftr_len, uint8_t *d_dst, uint64_t *d_dst_off, void *stream);

/*
 * Batching aggregator: concurrent single-message calls coalesced into device
 * batches (the reference's callers run BinaryConv.Do from many goroutines,
 * conv/j2t/conv_timing_test.go:76-99). dg_agg_do blocks the calling thread
 * until its message is converted, with the semantics of dg_j2t_do
 * (BinaryConv.Do, conv/j2t/conv.go:53-77); see dg_agg_create2 for when a
 * batch is converted. If out_cap is too small the call returns
 * DG_E_NOMEM with *out_len = the bytes needed. Thread-safe.
 */
int dg_agg_create(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, uint64_t flags, uint32_t max_batch,
                  uint32_t max_wait_us, dg_agg **out);
int dg_agg_do(dg_agg *agg, const uint8_t *json, size_t len, uint8_t *out, size_t out_cap, size_t *out_len,
              uint64_t *ret);
/* dg_agg_create with an explicit JSON capacity. Capacities are per caller
 * thread: every thread that calls owns a part of each device batch holding
 * up to max_batch messages and max_bytes JSON bytes (a message longer than
 * max_bytes is converted alone); a batch is sealed when one thread's part is
 * full, when a caller waits on it, or when its first message has waited
 * max_wait_us. dg_agg_create uses max_bytes = max(1 MiB, 512 B x max_batch).
 * The first 224 calling threads get a part each; further threads share the
 * last 32 parts under a per-part lock (no thread count converts alone).
 * Pinned host memory: every part that is in use holds ring x (8 x max_batch +
 * max_bytes + 64) bytes (ring = DG_AGG_RING, default 16, at most 24), e.g. 16
 * threads x 16 x (8 x 4096 + 2 MiB) = 520 MiB. On top of that, every batch
 * of the ring keeps buffers for the largest batch the registered parts can
 * make, P = 4 x (parts x max_bytes) + 128 x (parts x max_batch) bytes of
 * packed output: about P of pinned host memory and 5 P of device memory per
 * batch, ring x that in all. They are sized exactly (never regrown mid-run)
 * while ring x P <= 4 GiB (knob "exact_total"), else grown lazily to twice
 * the batch that needed them. E.g. 16 threads, max_batch 4096, max_bytes
 * 1 MiB: P = 72 MiB, ring 16: 1.15 GiB pinned + 5.8 GiB device. Size
 * max_batch / max_bytes for the caller threads the process runs. */
int dg_agg_create2(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, uint64_t flags, uint32_t max_batch,
                   uint64_t max_bytes, uint32_t max_wait_us, dg_agg **out);
/* Asynchronous form of dg_agg_do, for a caller with many requests in flight
 * (an event loop, or a goroutine pool behind one OS thread): dg_agg_submit
 * copies the JSON into the open batch and returns a ticket; dg_agg_wait
 * blocks until the ticket's batch is converted and copies its result out
 * (same results as dg_agg_do). Every ticket must be waited for exactly once,
 * and `json` must stay valid until then. With nonblock, dg_agg_submit
 * returns DG_E_AGAIN instead of blocking when no batch is open (a caller
 * that holds unwaited tickets must use it, and wait for its oldest ticket
 * before retrying: the next batch opens when the oldest one's callers have
 * taken their results). */
typedef struct dg_agg_ticket {
    void *batch;
    uint64_t gen;
    uint32_t idx;
    const uint8_t *json;
    size_t len;
} dg_agg_ticket;
int dg_agg_submit(dg_agg *agg, const uint8_t *json, size_t len, int nonblock, dg_agg_ticket *t);
int dg_agg_wait(dg_agg *agg, dg_agg_ticket *t, uint8_t *out, size_t out_cap, size_t *out_len, uint64_t *ret);
/* 1 when dg_agg_wait on the ticket would not block (its batch is converted),
 * else 0: an event loop takes its completions as they come. */
int dg_agg_ready(dg_agg *agg, const dg_agg_ticket *t);
/* batches flushed and messages converted so far */
int dg_agg_stats(dg_agg *agg, uint64_t *batches, uint64_t *msgs);
/* diagnostics: n <= 16 summed counters (ns unless noted) (flusher waiting for a seal,
 * for a free batch, issuing a batch; completer waiting for the header, for
 * the packed bytes; seal to issued; issued to done; callers blocked in
 * dg_agg_wait; dg_agg_drive: time in submit, in wait, and the count of
 * submits that met no open batch; the count of calls converted alone by
 * dg_j2t_do: longer than a part, or no part left for their thread; the
 * flusher's issue split in four: waiting for the parts' writers, buffers,
 * the gather launch, the conversion's launches).
 * An exclusive part (one of 224) belongs to a calling thread from its first
 * call until the thread exits; an exited thread's part goes to the next new
 * thread. */
int dg_agg_profile(dg_agg *agg, uint64_t *out, int n);
/* converts what is still queued, then stops the flusher (every ticket must
 * have been waited for) */
void dg_agg_destroy(dg_agg *agg);
/* Benchmark driver (the reference's b.RunParallel over Do,
 * conv/j2t/conv_timing_test.go:76-99): `threads` OS threads each convert a
 * contiguous share of the n messages through the aggregator with up to
 * `window` requests in flight, message i's result into
 * out[out_off[i] .. out_off[i+1]) with out_len[i], ret[i], and, if lat_ns,
 * its submit-to-result latency for every 8th message (0 for the others: the
 * clock is read for a sample of the calls only). *seconds = wall time of
 * the whole run. */
int dg_agg_drive(dg_agg *agg, const uint8_t *arena, const uint64_t *in_off, uint64_t n, int threads, int window,
                 uint8_t *out, const uint64_t *out_off, uint64_t *out_len, uint64_t *ret, uint32_t *lat_ns,
                 double *seconds);

/* The gateway binding: goroutines do not hold an OS
 * thread while their call converts. A Do submits without blocking
 * (dg_agg_submit nonblock), takes the ticket's generation
 * (dg_agg_ticket_gen) and parks on a Go channel for it; ONE poller thread
 * blocks in dg_agg_wait_gen, which returns once batches up to a newer
 * generation are converted (generations complete in order), and wakes the
 * goroutines of every generation up to it; each then calls dg_agg_wait,
 * which no longer blocks, to copy its result. Every ticket must be waited
 * for, from any thread. */
int dg_agg_wait_gen(dg_agg *agg, uint64_t after, uint32_t timeout_us, uint64_t *done);
uint64_t dg_agg_ticket_gen(const dg_agg_ticket *t);
/* aggregator knobs: "depth" (0 = off): also seal the open batch as soon as
 * it holds a message and fewer than depth batches are converting -- for
 * callers that park instead of blocking in dg_agg_wait, whose waits the
 * aggregator cannot see; "min_fill" (0 = off): the depth rule seals only a
 * batch of at least this many calls (many parked callers refill a batch
 * over a round trip: sealing at once keeps batches small); "max_wait_us":
 * the seal timer of dg_agg_create; "exact_total" (bytes, default 4 GiB):
 * the ring-wide budget for sizing batch buffers exactly (dg_agg_create2). */
int dg_agg_set_knob(dg_agg *agg, const char *name, int64_t value);
/* Benchmark driver for the gateway shape: `callers` logical callers, each
 * with ONE call in flight at a time (a goroutine in Do), multiplexed over
 * `workers` OS threads (the Go runtime's Ms) with the dg_agg_wait_gen poller
 * above; worker w serves messages [w n / workers, (w + 1) n / workers) in
 * order, each runnable caller taking the next one (workers is clamped to
 * min(workers, callers, n): a worker needs callers for its range). Outputs as
 * dg_agg_drive; stats (optional, 8 u64): parks, submits retried for want of
 * room, poller wake-ups, callers, then ns summed over the workers in
 * dg_agg_wait, in dg_agg_submit, idle, and in all. */
int dg_agg_gateway_drive(dg_agg *agg, const uint8_t *arena, const uint64_t *in_off, uint64_t n, int workers,
                         int callers, uint8_t *out, const uint64_t *out_off, uint64_t *out_len, uint64_t *ret,
                         uint32_t *lat_ns, double *seconds, uint64_t *stats);

/* dg_j2t_batch_host for large host batches: the batch is streamed in
 * `chunks` pieces through 3 stream-private buffer sets, so the upload of
 * chunk k+1, the kernels of chunk k and the download of chunk k-1 overlap,
 * all issued from C. json, in_off, out, out_off and ret should be pinned
 * (hipHostMalloc) for the copies to be asynchronous. Same outputs and
 * DG_E_NOMEM/out_need contract as dg_j2t_batch_host; json needs no padding. */
int dg_j2t_pipeline_host(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *json,
                         const uint64_t *in_off, uint64_t n, uint64_t flags, uint32_t chunks, uint8_t *out,
                         uint64_t out_cap, uint64_t *out_off, uint64_t *ret, uint64_t *out_need);

/*
 * t2j: Thrift binary -> JSON (the reverse path, conv/t2j). Replaces
 * BinaryConv.Do / DoInto (conv/t2j/conv.go:50-95 over impl.go:74-468) for
 * the options in dgj2t_defs.h DG_T2J_* (the Go-side ones -- HTTP mapping,
 * ConvertException, EnableThriftBase -- stay on the Go host).
 *
 * dg_desc_attach_t2j uploads the descriptor's t2j side table (the JSON key
 * text per field, include/dgj2t_desc.h dg_t2j_*) once; the t2j entry points
 * need it. Status words: 0, DG_T2J_E_* | pos << 8 | value << 40 (pos = the
 * Thrift read offset), or DG_ST_OUT_OVERFLOW with *out_len = bytes needed
 * (device entry point only; the host entry point reruns those itself).
 * Nesting deeper than the fast kernel's LDS frames is rerun on device with
 * 4096 frames per message; deeper still is DG_T2J_E_DEPTH.
 */
int dg_desc_attach_t2j(dg_desc *desc, const void *side, size_t len);
/* the slot size the host entry point gives a message of len Thrift bytes:
 * 3 len + 64 rounded up to 128 (a guess: JSON has no fixed bound over Thrift;
 * larger outputs overflow and are rerun with their exact size) */
uint64_t dg_t2j_slot_bound(uint64_t len);
/* device buffers, stream-ordered, async; arena readable 16 bytes past the
 * last message; d_out_off 8-aligned slots */
int dg_t2j_batch_device(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *d_thrift,
                        const uint64_t *d_in_off, uint64_t n, uint64_t opts, uint8_t *d_out,
                        const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret, void *stream);
/* The same with the batch's longest Thrift message (0 = unknown): the kernel
 * gives short messages full waves and ~1 KB ones sparse waves (t2j-c2 +4 %,
 * t2j-c3 +5 % over the size-blind launch). */
int dg_t2j_batch_device_ml(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *d_thrift,
                           const uint64_t *d_in_off, uint64_t n, uint64_t opts, uint8_t *d_out,
                           const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret, void *stream,
                           uint64_t max_len);
/* host buffers, synchronous: JSON packed back to back into out (out_off[n+1]);
 * DG_E_NOMEM with *out_need when out_cap is too small */
int dg_t2j_batch_host(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *thrift,
                      const uint64_t *in_off, uint64_t n, uint64_t opts, uint8_t *out, uint64_t out_cap,
                      uint64_t *out_off, uint64_t *ret, uint64_t *out_need);

/* dg_t2j_batch_device_ml / dg_t2j_batch_host with the device part of the Go-side options
 * device part (dgj2t_defs.h DG_T2J_CONVERT_EXC, DG_T2J_SKIP_RESP_BASE): aux
 * (n u64, device resp. host memory) receives each message's response-base
 * span when DG_T2J_SKIP_RESP_BASE is set (may be NULL otherwise); a
 * DG_T2J_E_EXCEPTION message keeps its JSON in out. */
int dg_t2j_batch_device_aux(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *d_thrift,
                            const uint64_t *d_in_off, uint64_t n, uint64_t opts, uint8_t *d_out,
                            const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret, uint64_t *d_aux,
                            void *stream, uint64_t max_len);
int dg_t2j_batch_host_aux(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *thrift,
                          const uint64_t *in_off, uint64_t n, uint64_t opts, uint8_t *out, uint64_t out_cap,
                          uint64_t *out_off, uint64_t *ret, uint64_t *out_need, uint64_t *aux);
/* ... and EnableHttpMapping's response side (DG_T2J_HM; conv/t2j/impl.go:
 * 132-142, 296-306, writeHttpValue 515-588; HandleRequires' mapped unsets):
 * a mapped field of the root struct or of a struct that is a root field's
 * value stops the message with DG_T2J_E_CALLBACK and a 16-byte record in out
 * (dgj2t_defs.h). The host runs writeHttpValue (dynamicgo_amd/t2j.py) and
 * converts the message again with its answers: ans_tab (n entries, device
 * resp. host memory) indexes one byte per answer in the answer bytes, consumed
 * in the order the stops come. cb: only ans_tab, bytes and len are read. */
int dg_t2j_batch_device_cb(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *d_thrift,
                           const uint64_t *d_in_off, uint64_t n, uint64_t opts, uint8_t *d_out,
                           const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret, uint64_t *d_aux,
                           const dg_cb_entry *d_ans, const uint8_t *d_ans_bytes, void *stream, uint64_t max_len);
int dg_t2j_batch_host_cb(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *thrift,
                         const uint64_t *in_off, uint64_t n, uint64_t opts, uint8_t *out, uint64_t out_cap,
                         uint64_t *out_off, uint64_t *ret, uint64_t *out_need, uint64_t *aux, const dg_cb_tables *cb);

/* Timing helper for benchmarks: launch the device batch `iters` times on the
 * context stream bracketed by HIP events; returns total milliseconds of GPU
 * time in *ms (events are recorded on the stream the kernels run on). */
int dg_bench_device(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, const uint8_t *d_json,
                    const uint64_t *d_in_off, uint64_t n, uint64_t flags, uint8_t *d_out,
                    const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret, int iters,
                    float *ms);

#ifdef __cplusplus
}
#endif
#endif /* DGJ2T_H */
