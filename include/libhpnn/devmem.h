/*
 * libhpnn caching device allocator.
 *
 * The engines allocate their device state per nn_train_kernel / nn_run_kernel call
 * (weights, momentum, split-K slabs, activations, the resident dataset); the tutorial
 * workflow calls train_nn / run_nn in loops, and a large hipMalloc costs milliseconds.
 * Freed blocks go to per-device, size-class free lists and are handed out again on the
 * next request of the same class; the reference allocated and freed on every call
 * (cuda_ann.cu:192-331).  A free synchronises the owning device first (hipFree
 * semantics: no kernel can still be using a block that is handed out again).  When
 * hipMalloc fails the device's cached blocks are released and the request retried.
 * HPNN_DEVMEM_CACHE=0 disables caching (straight hipMalloc / hipFree).
 */
#ifndef LIBHPNN_DEVMEM_H
#define LIBHPNN_DEVMEM_H
#include <hip/hip_runtime_api.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

hipError_t hpnn_dev_malloc_raw(void **p, size_t bytes);
hipError_t hpnn_dev_free(void *p);
/* release every cached block (all devices) */
void hpnn_dev_trim(void);
/* bytes handed out, bytes cached, cache hits, hipMalloc calls */
void hpnn_dev_stats(size_t *in_use, size_t *cached, size_t *hits, size_t *misses);

#ifdef __cplusplus
}
template <class T>
static inline hipError_t hpnn_dev_malloc(T **p, size_t bytes) {
    return hpnn_dev_malloc_raw((void **)p, bytes);
}
#endif
#endif
