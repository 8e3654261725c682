/* libhpnn internal runtime helpers (not part of the public C API). */
#ifndef HPNN_RUNTIME_INTERNAL_H
#define HPNN_RUNTIME_INTERNAL_H
#include <libhpnn.h>

nn_runtime *hpnn_rt_get(void);
int hpnn_rt_device(UINT gpu);
hipStream_t hpnn_rt_stream(UINT gpu, UINT idx);
BOOL hpnn_rt_gpu_available(void);
void hpnn_rt_probe_memory_model(void);
/* implemented by the GPU engine: frees device buffers still referenced */
void hpnn_rt_release_device_state(void);

/* line reader that accepts arbitrarily long lines; returns NULL on EOF */
char *hpnn_readline(FILE *fp, char **buf, size_t *cap);

#endif
