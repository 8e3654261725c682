/*
 * libhpnn xGMI all-reduce: peer-to-peer sum all-reduce for small buffers between the
 * GPUs of one node (csrc/dist/xgmi_ar.hip).
 *
 * Why: MNIST's whole gradient is 437 KB.  A ring all-reduce (RCCL) of that size over
 * 8 MI355X is latency-bound -- 2(N-1) = 14 dependent hops -- while each GPU has a direct
 * xGMI link to every other GPU.  Here every rank publishes its buffer in device memory
 * that every peer maps (hipIpc handles), and one kernel per rank runs either
 *   one-shot: copy in -> flag barrier -> read the slice from all N buffers and sum them
 *             in rank order (identical bits on every rank, deterministic); or
 *   two-shot: copy in -> barrier -> reduce this rank's 1/N shard from all N buffers ->
 *             barrier -> read the N-1 reduced shards from their owners (each xGMI link
 *             carries 2/N of the buffer instead of all of it).
 * Auto choice (HPNN_XAR_MODE=0): two-shot from 4 ranks and 64 KiB, else one-shot
 * (HPNN_XAR_MODE=1 / 2 force one).  Consecutive calls alternate between two halves of
 * the buffer, so no closing barrier is needed before a buffer is refilled.
 *
 * Graph capture: the barrier epochs live in device memory and are advanced by the
 * kernel itself, so a captured launch replays correctly any number of times.
 * Failure: every spin wait is bounded (HPNN_XAR_TIMEOUT_MS, default 20000); a peer that
 * never arrives sets the error word instead of hanging the GPU, and
 * hpnn_xar_status reports it.
 *
 * Usage (one process per GPU): c = hpnn_xar_create(rank, world, max_bytes);
 * hpnn_xar_handles(c, h) -> exchange world * HPNN_XAR_HANDLE_BYTES bytes (any
 * bootstrap, e.g. torch.distributed all_gather); hpnn_xar_open(c, all);
 * hpnn_xar_all_reduce_f32(c, in, out, count, stream).
 */
#ifndef LIBHPNN_XAR_H
#define LIBHPNN_XAR_H
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HPNN_XAR_MAX_RANKS 8
#define HPNN_XAR_MAX_BLOCKS 256
#define HPNN_XAR_MAX_SEGS 4
#define HPNN_XAR_HANDLE_BYTES 128

typedef struct hpnn_xar hpnn_xar;

hpnn_xar *hpnn_xar_create(int rank, int world, size_t max_bytes);
/* this rank's IPC handles (HPNN_XAR_HANDLE_BYTES bytes) */
int hpnn_xar_handles(hpnn_xar *c, void *out);
/* all ranks' handles, rank r at r * HPNN_XAR_HANDLE_BYTES */
int hpnn_xar_open(hpnn_xar *c, const void *all);
size_t hpnn_xar_max_bytes(const hpnn_xar *c);
/* out = sum over ranks of in (float32, count % 4 == 0, count * 4 <= max_bytes);
 * in == out allowed */
int hpnn_xar_all_reduce_f32(hpnn_xar *c, const float *in, float *out, long count, hipStream_t stream);
/* out = sum over ranks of [seg_0 | seg_1 | ...], segment j being the LOCAL sum of S_j
 * slabs src_j + s * stride_j (count_j floats each, multiples of 4): the split-K slab
 * reduction of the weight gradients happens inside the all-reduce's copy-in phase */
typedef struct {
    const float *src;
    long stride; /* floats between slabs */
    int S;       /* slabs */
    long count;  /* floats */
} hpnn_xar_seg;
int hpnn_xar_all_reduce_slabs_f32(hpnn_xar *c, const hpnn_xar_seg *segs, int nseg, float *out, hipStream_t stream);
/* the same all-reduce followed, in the same kernel, by every layer's optimizer step on the
 * reduced gradient (the math of hpnn_sgd_update_multi: g * scale, BP or BPM with momentum
 * alpha, FP32 master W32 / V32, BF16 copies Wbf [N x K], Wt [K x N] and, optionally,
 * the fragment-major Wf).  Layer l covers floats [sum_{j<l} N_j K_j, + N_l K_l) of the
 * output; the layers must cover it exactly.  Saves the separate update launch of a
 * data-parallel step; every rank applies the same bits. */
#define HPNN_XAR_MAX_LAYERS 8
typedef struct {
    float *W32;
    float *V32; /* NULL without momentum */
    void *Wbf;
    void *Wt;
    void *Wf; /* may be NULL */
    int N, K;
} hpnn_xar_upd_layer;
int hpnn_xar_all_reduce_slabs_update_f32(hpnn_xar *c, const hpnn_xar_seg *segs, int nseg, float *out,
                                         const hpnn_xar_upd_layer *layers, int nl, float lr, float alpha, float scale,
                                         int momentum, hipStream_t stream);
/* in-place form: a producer kernel writes this rank's contribution to the NEXT call
 * straight into the buffer -- at buf + half when *sel is even, at buf when odd (read *sel
 * on the device, in stream order: graph replays stay correct) -- and
 * hpnn_xar_reduce_local_update_f32 then runs the barrier, the peer sums and the step with
 * no copy-in phase.  The double-buffer argument is the copy-in's: the producer runs after
 * this rank's previous call, whose barrier no peer passes before finishing the call before. */
int hpnn_xar_local(hpnn_xar *c, float **buf, long *half, const unsigned int **sel);
int hpnn_xar_reduce_local_update_f32(hpnn_xar *c, long count, float *out, const hpnn_xar_upd_layer *layers, int nl,
                                     float lr, float alpha, float scale, int momentum, hipStream_t stream);
/* the communicator as seen by a kernel that runs the one-shot protocol itself (the fused
 * data-parallel first-layer gradient, kernels_g0.hip): every rank's buffer (two halves of
 * `half` floats) and signal block, this rank's per-workgroup epochs.  Workgroup b of every
 * rank owns the same elements; the kernel advances ep[b], stores into half (ep[b] & 1) of its
 * own buffer, waits for its stores, writes flag A of (b, rank) on every peer, waits for flag A
 * of (b, p) from every peer, then reads the peers' halves.  An instance used this way must not
 * also serve hpnn_xar_all_reduce* calls (their workgroups own other elements). */
typedef struct {
    float *buf[HPNN_XAR_MAX_RANKS];
    unsigned int *sig[HPNN_XAR_MAX_RANKS];
    long half;
    unsigned int *ep;
    int rank, world;
    unsigned long long timeout; /* wall-clock ticks */
} hpnn_xar_view;
#define HPNN_XAR_FLAG_A(sig, b, r) ((sig) + (long)(b) * HPNN_XAR_MAX_RANKS + (r))
#define HPNN_XAR_FLAG_B(sig, b, r) ((sig) + (long)(HPNN_XAR_MAX_BLOCKS + (b)) * HPNN_XAR_MAX_RANKS + (r))
#define HPNN_XAR_ERROR_WORD (2 * HPNN_XAR_MAX_BLOCKS * HPNN_XAR_MAX_RANKS)
int hpnn_xar_view_get(hpnn_xar *c, hpnn_xar_view *v);
/* 0 healthy, -1 a barrier timed out on this rank (a peer never arrived) */
int hpnn_xar_status(hpnn_xar *c);
/* the error word copied into *dst (pinned host memory) on `stream` without waiting; non-zero
 * once the event after it completes = hpnn_xar_status's -1 */
int hpnn_xar_status_enqueue(hpnn_xar *c, unsigned int *dst, hipStream_t stream);
/* collective self-test, run by every rank right after hpnn_xar_open: all-reduces known
 * rank-dependent vectors (every partial sum exact in FP32, so any summation order gives
 * the same bits) at a one-shot size and at the full buffer size, twice each so both
 * buffer halves are used, and compares the result on the device.  Returns 0 when this
 * rank received exactly the expected sums, -1 on a wrong element (peer writes not visible
 * over the links: coherence / mapping fault), -2 on a barrier timeout, -3 on a HIP error.
 * Every rank must call it (it is a collective); callers then agree across ranks (MIN of
 * the results) before the all-reduce is used. */
int hpnn_xar_self_test(hpnn_xar *c, hipStream_t stream);
void hpnn_xar_destroy(hpnn_xar *c);

#ifdef __cplusplus
}
#endif
#endif
