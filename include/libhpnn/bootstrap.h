/*
 * libhpnn launcher bootstrap: a host-side all-gather of small blobs between the processes
 * of one node (one process per GPU, launched by torchrun or any launcher that exports
 * RANK / WORLD_SIZE / LOCAL_RANK), through files in a directory every process sees.
 *
 * Used by the native (non-Python) multi-process data parallelism of nn_train_kernel to
 * exchange the xGMI all-reduce IPC handles, the RCCL unique id and per-epoch statistics;
 * the Python path uses torch.distributed instead.  Directory: HPNN_BOOT_DIR, else
 * $TMPDIR (or /tmp) / hpnn_boot_<MASTER_ADDR>_<MASTER_PORT>_<TORCHELASTIC_RUN_ID>.
 * Files older than 2 minutes before this process started are ignored (a previous job
 * with the same address and port).  Every wait is bounded (HPNN_BOOT_TIMEOUT_S, 120 s).
 */
#ifndef LIBHPNN_BOOTSTRAP_H
#define LIBHPNN_BOOTSTRAP_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* rank / world of the launcher environment (0 / 1 without one) */
int hpnn_boot_rank(void);
int hpnn_boot_world(void);
/* all[r * n .. r * n + n) = rank r's `mine` (n bytes); every rank calls with the same n and
 * in the same order; returns 0 or < 0 (timeout, I/O error) */
int hpnn_boot_allgather(const void *mine, size_t n, void *all);
/* two barriers, then rank 0 removes the exchange files every rank has finished reading */
void hpnn_boot_finish(void);

#ifdef __cplusplus
}
#endif
#endif
