/*
 * libhpnn communication layer (MI355X-native): RCCL over xGMI.
 *
 * Replaces the reference's inline MPI collectives (MPI_Allgather of
 * activations / deltas / weights, MPI_Allreduce of scalars, MPI_Bcast of weights,
 * MPI_Send/Recv bail-out) and its CUDA hub copies (cuda_ann.cu EXP model) with one
 * communicator object per GPU:
 *   - multi-process (one process per GPU, torch.distributed launch): the unique id
 *     is created on rank 0 (hpnn_comm_unique_id) and shipped by the caller's
 *     bootstrap (torch.distributed / a file / a socket), then hpnn_comm_init_rank;
 *   - single process driving G GPUs: hpnn_comm_init_all.
 * RCCL is resolved at run time with dlopen (the torch-ROCm wheel in the same
 * process may already hold its own librccl; dlopen by soname reuses it).
 *
 * Overlap: every collective issued with *_async runs on the communicator's own
 * side stream.  It waits (hipEvent) only for the work already enqueued on the
 * caller's compute stream, so it overlaps whatever the compute stream does next;
 * hpnn_comm_join makes the compute stream wait for all outstanding collectives.
 * Event record / wait are stream-capturable, so a whole data-parallel step can be
 * captured in a HIP graph (fork/join of the side stream).
 *
 * Return values: 0 success, < 0 error (message on stderr through NN_ERROR).
 */
#ifndef LIBHPNN_COMM_H
#define LIBHPNN_COMM_H
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HPNN_COMM_ID_BYTES 128

typedef struct hpnn_comm hpnn_comm;

typedef enum {
    HPNN_DT_F32 = 0,
    HPNN_DT_F64 = 1,
    HPNN_DT_BF16 = 2,
    HPNN_DT_I32 = 3,
    HPNN_DT_U8 = 4,
} hpnn_comm_dtype;

typedef enum {
    HPNN_OP_SUM = 0,
    HPNN_OP_MAX = 1,
    HPNN_OP_MIN = 2,
} hpnn_comm_op;

/* 1 if librccl could be loaded with every symbol the layer needs */
int hpnn_comm_available(void);
/* rank 0: fill id[HPNN_COMM_ID_BYTES] (ncclGetUniqueId) */
int hpnn_comm_unique_id(unsigned char *id);
/* one communicator for this process' GPU `device` (multi-process mode) */
hpnn_comm *hpnn_comm_init_rank(const unsigned char *id, int nranks, int rank, int device);
/* single process, G devices: comms[g] for devs[g] */
int hpnn_comm_init_all(hpnn_comm **comms, int G, const int *devs);
void hpnn_comm_destroy(hpnn_comm *c);
int hpnn_comm_rank(const hpnn_comm *c);
int hpnn_comm_size(const hpnn_comm *c);

/* in-order collectives on `stream` (in place when send == recv) */
int hpnn_comm_all_reduce(hpnn_comm *c, const void *send, void *recv, long count, hpnn_comm_dtype dt,
                         hpnn_comm_op op, hipStream_t stream);
int hpnn_comm_broadcast(hpnn_comm *c, const void *send, void *recv, long count, hpnn_comm_dtype dt, int root,
                        hipStream_t stream);
/* recv holds nranks * count elements, rank r's block at r * count */
int hpnn_comm_all_gather(hpnn_comm *c, const void *send, void *recv, long count, hpnn_comm_dtype dt,
                         hipStream_t stream);
/* send holds nranks * count elements; recv gets the reduced block of this rank */
int hpnn_comm_reduce_scatter(hpnn_comm *c, const void *send, void *recv, long count, hpnn_comm_dtype dt,
                             hpnn_comm_op op, hipStream_t stream);
/* grouped launch of several collectives (single-process multi-GPU must group the
 * per-device calls) */
int hpnn_comm_group_start(void);
int hpnn_comm_group_end(void);

/* overlapped sum all-reduce on the side stream (see header comment) */
int hpnn_comm_all_reduce_async(hpnn_comm *c, void *buf, long count, hpnn_comm_dtype dt, hipStream_t compute);
/* general fork: the side stream, ordered after what `compute` has enqueued so far; the caller
 * enqueues kernels and collectives on it, then hpnn_comm_fork_done so hpnn_comm_join covers
 * them.  NULL on failure. */
hipStream_t hpnn_comm_fork(hpnn_comm *c, hipStream_t compute);
int hpnn_comm_fork_done(hpnn_comm *c);
/* compute stream waits for every collective issued with *_async so far */
int hpnn_comm_join(hpnn_comm *c, hipStream_t compute);

/* route *_async float32 sum all-reduces of at most max_bytes through the one-shot xGMI
 * all-reduce x (include/libhpnn/xar.h; NULL detaches); larger ones stay on RCCL */
struct hpnn_xar;
int hpnn_comm_set_xar(hpnn_comm *c, struct hpnn_xar *x, size_t max_bytes);

/* failure detection: 0 healthy, < 0 the communicator reported an asynchronous error
 * (a peer died, a link failed) -- the caller should abort it */
int hpnn_comm_check(hpnn_comm *c);
/* abort all outstanding work of a failed communicator (ncclCommAbort) */
void hpnn_comm_abort(hpnn_comm *c);

/* all ranks agree on a status: returns the MIN over ranks of `ok` (1 = all ok),
 * the collective replacement of the reference's MPI bail-out (ann.c:237-249).
 * Synchronises `stream`. */
int hpnn_comm_all_ok(hpnn_comm *c, int ok, hipStream_t stream);

/* fault injection for tests: HPNN_FAULT=<site>:<n>[,<site>:<n>] makes the n-th
 * (1-based) event at `site` fail (sites: comm, sample, load, nan, stop; handoff: a fused
 * split-K launch reports a timed-out wait; digest / weights: one replica's weight digest /
 * weights differ, in train_nn / bench.py); returns 1
 * when it fires */
int hpnn_fault_hit(const char *site);

#ifdef __cplusplus
}
#endif
#endif
