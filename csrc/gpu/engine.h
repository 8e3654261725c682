/*
 * libhpnn GPU engines (HIP, gfx950) -- host-side interface.
 *
 * Two engines live behind this header:
 *   online  : the reference's batch-1, iterate-to-convergence training
 *              in FP64.  The WHOLE per-sample convergence loop
 *             (train step, re-forward, error, argmax, stop test) runs inside
 *             one persistent single-workgroup kernel, so there is no host
 *             round trip per iteration (the reference synchronised the host
 *             on every iteration: ann.c:2329-2332, cuda_ann.cu:1294).
 *   batched : minibatch SGD / momentum with MFMA GEMMs (BF16 in, FP32
 *             accumulate, FP32 master weights) or FP32/FP64 MFMA.
 */
#ifndef HPNN_GPU_ENGINE_H
#define HPNN_GPU_ENGINE_H
#include <libhpnn/ann.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- online (reference semantics) ---- */
/* uploads the host weights if the device copy is stale */
BOOL hpnn_gpu_online_prepare(kernel_ann *k, UINT gpu);
DOUBLE hpnn_gpu_train_sample(kernel_ann *k, nn_type type, nn_train train, const DOUBLE *in,
                             const DOUBLE *out, DOUBLE lr, DOUBLE alpha, DOUBLE delta, UINT *n_iter,
                             BOOL *ok, DOUBLE *init_err, BOOL *first_ok);
/* forward only; result copied to k->output.vec (host) */
BOOL hpnn_gpu_forward(kernel_ann *k, nn_type type, const DOUBLE *in);
/* device weights -> host master copy (no-op if host is current) */
void hpnn_gpu_sync_host(kernel_ann *k);
/* TRUE once a device state was lost (a grid barrier timed out mid-sample): the caller
 * stops training; the host weights are the last consistent ones */
BOOL hpnn_gpu_failed(const kernel_ann *k);
/* online slot layout (pure): n_gpu, -S streams, runtime memory model, HPNN_ONLINE_SLOTS */
int hpnn_online_slot_plan(int n_gpu, int n_streams, int mem_model, int env_slots, int *spd);
/* host master copy changed: mark device copy stale */
void hpnn_gpu_mark_host_dirty(kernel_ann *k);

/* ---- batched ---- */
typedef struct {
    nn_type type;
    nn_train train;
    nn_dtype dtype;
    UINT batch;
    UINT epochs;
    DOUBLE lr;
    DOUBLE alpha;
    UINT seed;
    UINT n_gpu;       /* data-parallel replicas driven by this process */
    BOOL resume;      /* BPM: start from the momentum in k->dw (exact resume)  */
    UINT epoch0;      /* epochs completed before this call (metrics numbering) */
    UINT tp;          /* 1: row-sharded tensor parallelism ([parallel] tp; f64 / f32 / bf16) */
} hpnn_batched_opts;

typedef struct {
    DOUBLE last_loss;   /* mean loss of the last minibatch            */
    DOUBLE epoch_loss;  /* mean loss over the last epoch              */
    UINT64 samples;     /* samples processed                          */
    DOUBLE seconds;     /* wall time spent in the training loop       */
    UINT correct;       /* argmax hits in the last epoch              */
} hpnn_batched_stats;

/* X: n x n_in, T: n x n_out (host, row-major FP64). Weights are read from
 * and written back to the host kernel; with BPM the final momentum is written to
 * k->dw (allocated if needed) so that nn_dump_state can save it. */
BOOL hpnn_gpu_train_batched(kernel_ann *k, const DOUBLE *X, const DOUBLE *T, UINT n,
                            const hpnn_batched_opts *o, hpnn_batched_stats *st);
/* the same with every hidden layer's rows sharded over the ranks (tp_engine.cpp): ranks =
 * HPNN_LOOPBACK_RANKS threads on GPU 0, the launcher's processes, or o->n_gpu GPUs */
BOOL hpnn_gpu_train_tp(kernel_ann *k, const DOUBLE *X, const DOUBLE *T, UINT n, const hpnn_batched_opts *o,
                       hpnn_batched_stats *st);
/* batched inference: Y = net(X), n x n_out (host) */
BOOL hpnn_gpu_infer_batched(kernel_ann *k, nn_type type, nn_dtype dtype, const DOUBLE *X, UINT n,
                            DOUBLE *Y);

/* CPU batched engine (FP64 oracle for the batched semantics) */
BOOL hpnn_cpu_train_batched(kernel_ann *k, const DOUBLE *X, const DOUBLE *T, UINT n,
                            const hpnn_batched_opts *o, hpnn_batched_stats *st);
/* one minibatch step on the CPU: returns mean loss before the update */
DOUBLE hpnn_cpu_batched_step(kernel_ann *k, nn_type type, const DOUBLE *X, const DOUBLE *T, UINT b,
                             DOUBLE lr, BOOL momentum, DOUBLE alpha, UINT *hits /* may be NULL: += argmax hits */);

#ifdef __cplusplus
}
#endif
#endif
