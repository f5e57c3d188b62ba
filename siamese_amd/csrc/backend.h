// backend.h -- the only interface between the host control plane and the
// device.  libsiamese_amd.so implements it with HIP on gfx950
// (backend_hip.hip).  A host simulation of the same contract exists ONLY for
// the CPU test suite (tests/hostsim/), never in the shipped library.
#pragma once

#include "ops.h"
#include <cstddef>
#include <cstdint>

namespace sgpu {

/// Initialise the device (HIP device index; <0 = current).  Returns false
/// with a message in *err when no usable MI355X device exists.
bool be_init(int device, const char** err);
const char* be_name();

void* be_dev_alloc(size_t bytes);
void be_dev_free(void* p);
void* be_host_alloc(size_t bytes);   // page-locked
/// Page-locked, mapped and coherent host memory: kernels read and write it
/// directly (zero-copy uploads, k_hostcopy downloads), and a buffer rewritten
/// between submissions is never seen stale through a device cache.
void* be_host_alloc_mapped(size_t bytes);
/// The device's address of page-locked host memory (kernels read it over
/// the bus: zero-copy).
void* be_host_device_ptr(void* host);
void be_host_free(void* p);

// All transfers and launches are asynchronous on the engine's stream.
void be_h2d(void* dst, const void* src, size_t bytes);
void be_d2h(void* dst, const void* src, size_t bytes);
void be_memset(void* dst, int value, size_t bytes);
/// Copies between device memory and page-locked host memory (be_host_alloc):
/// small totals run as one kernel on the engine's stream (no copy-engine
/// hand-off, whose cross-queue wait costs more than the bytes on the
/// latency-bound single-stream path), large ones as DMA.
struct BeCopy
{
    uint64_t dst, src;
    uint64_t bytes;
};
constexpr unsigned kBeCopyMax = 8;   // ranges per be_copy_pinned call
void be_copy_pinned(const BeCopy* ranges, unsigned count, bool toDevice);
/// The same ranges with a device-readable copy of the list (devList: each
/// range's host side as the device addresses it, be_host_device_ptr), so
/// that any number of small ranges takes one kernel launch; null devList, or
/// ranges too large for a kernel, fall back to be_copy_pinned.
void be_copy_list(const BeCopy* ranges, const void* devList, unsigned count, bool toDevice);

/// One wave per (descriptor, kIngestChunkBytes chunk): maxBytes is the
/// largest hdrLen + bytes among the descriptors (sizes the grid).
/// blocks: the k_ingest block table (nblocks entries, descriptor << 4 |
/// 4-symbol group of its run), or null for runs of one (one per wave).
void be_launch_ingest(const IngestDesc* descs, uint32_t count, uint32_t maxBytes, const uint32_t* blocks = nullptr,
                      uint32_t nblocks = 0);
/// `stream`: the instruction words of every segment (see ExecItem).
/// `acct`: device counter the executor adds the reference's source bytes of
/// the terms it expands itself (sum updates, LDPC picks) to (ops.h).
/// `maxWindow`: the largest OP_ROWS window (entries) among the launched
/// segments, kNoRows when none has a row batch (sizes the LDS stage).
/// `results`: the submission's result words, which gate the rows of an
/// OP_ROWS batch whose GfOp.termBegin is non-zero (1 + the word; a zero word
/// skips the rows: a chained device elimination that failed, ops.h GeDesc).
void be_launch_exec(const void* stream, const ExecItem* items, uint32_t count, uint64_t* acct,
                    const uint32_t* results, uint32_t maxWindow);
/// Wide rows' LDPC picks (ops.h LdpcItem), one workgroup per item; adds the
/// reference's source bytes of the picks (min(len, n) each) to acct[0].
void be_launch_ldpc(const LdpcItem* items, uint32_t count, uint64_t* acct);
/// The triangular solves (reference SiameseDecoder.cpp:1065-1238), one
/// workgroup per SolveItem: every tile first solves bytes 0..3 of its rows
/// to learn the recovered lengths, the tile-0 item writes them to `results`
/// and adds acct[0] += the reference's source bytes of each
/// back-substitution step the solve completes (:1131-1212), acct[1] += the
/// recovered bytes it outputs.  maxRows: largest m among the solves (sizes
/// the LDS staging).
void be_launch_solve(const SolveDesc* solves, const SolveRow* rows, const uint8_t* coef, uint32_t* results,
                     const SolveItem* items, uint32_t count, uint32_t maxRows, uint64_t* acct,
                     uint32_t solveBegin, uint32_t solveCount);

/// Device recovery-matrix generation + elimination (ops.h GeDesc): one job
/// per desc, its input at in + desc.in, its output in results + desc.result;
/// a kGeChained job that succeeds also writes its solve's coefficients
/// (coef + solveCoef) and permutes its SolveRows (rows + solveRow).  Reads
/// nothing any other launch of the flush writes.  It may run beside the
/// launches queued after it until be_join_ge(), after which every launch
/// (and the results' download) sees its outputs.  maxRows / maxCols: the
/// largest job of the launch (sizes its LDS).  head (or null): a pinned H2D
/// copy that brings the jobs' inputs, rows and coefficients into place, run
/// ahead of them on their own stream (beside the codec stream's copies); it
/// must not overlap anything the codec stream writes or copies.
/// rowsIn (or null: rows): where a chained job reads its solve rows before it
/// writes them to `rows` in pivot order; with descs, in and rowsIn in mapped
/// pinned memory and no head, the jobs need no copy at all.
void be_launch_ge(const GeDesc* descs, const uint8_t* in, uint32_t count, uint32_t* results, SolveRow* rows,
                  uint8_t* coef, uint32_t maxRows, uint32_t maxCols, const BeCopy* head, bool side = true,
                  const SolveRow* rowsIn = nullptr);
/// The other arrangement: with side = false the jobs (and their head copy)
/// run in order on the codec stream, and this puts the rest of the upload
/// (`rest`, or null) and k_ingest (be_launch_ingest's arguments) on the side
/// stream beside them; be_join_ge joins it.
void be_side_upload_ingest(const BeCopy* rest, const IngestDesc* descs, uint32_t count, uint32_t maxBytes,
                           const uint32_t* blocks, uint32_t nblocks);
void be_join_ge();

/// Block until all queued work has finished.  Returns false on a device fault.
bool be_sync();

/// A marker after all work queued so far.  be_fence_wait blocks (sleeping,
/// not spinning) until the device has passed it, returns false on a device
/// fault, and releases it.  The launcher thread creates fences, the
/// completer thread waits for them.
void* be_fence();
/// spinUs: poll this long before sleeping (latency-bound small flushes);
/// sleepPoll: poll with short sleeps instead of the runtime's blocking wait,
/// which spins on the core first (large flushes on a CPU-quota-bound host).
bool be_fence_wait(void* fence, unsigned spinUs, bool sleepPoll);

/// Transfer streams beside the codec stream (end-to-end packet flows).
/// be_stage_h2d copies host -> device on the staging stream right away (the
/// caller guarantees that no unfinished submission touches dst) and returns
/// a mark; be_wait_mark makes the codec stream wait for it on the device
/// (the host never blocks); be_mark_release recycles it once that wait has
/// been queued.  Null mark: the copy could not be queued.
void* be_stage_h2d(void* dst, const void* src, size_t bytes);
void be_wait_mark(void* mark);
void be_mark_release(void* mark);
/// Gather on the gather stream: upload `count` ingest descriptors (from
/// pinned descsHost to descsDev), pack their sources into devStage and copy
/// `bytes` of it to hostOut, without waiting (not even for the gather
/// stream).  Returns two marks: *packed is passed once the sources have been
/// read (be_wait_mark / be_mark_release, like a staging mark), *landed once
/// hostOut holds the bytes (be_mark_sync).  False if it could not be queued.
bool be_gather(const IngestDesc* descsHost, void* descsDev, uint32_t count, const void* devStage,
               void* hostOut, size_t bytes, void** packed, void** landed);
/// Block until the device has passed `mark`, then recycle it; false on a
/// device fault.
bool be_mark_sync(void* mark);

/// Device-time accounting: every executor/solve launch is bracketed with
/// events; these return the accumulated milliseconds since the last reset.
/// Kernel classes of the per-launch device timing.
enum BeKernel { kBeIngest, kBeExec, kBeLdpc, kBeSolve, kBeGe, kBeKernelKinds };
void be_timing_enable(bool on);
/// Device milliseconds of one kernel class since the last reset
/// (be_timing_exec_ms is kBeExec's).
double be_timing_kernel_ms(BeKernel kind);
void be_timing_reset();
double be_timing_exec_ms();
double be_timing_total_ms();

} // namespace sgpu
