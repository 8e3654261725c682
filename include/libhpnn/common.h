/*
 * libhpnn (MI355X-native) -- common definitions shared by the C API, the
 * native engines and the CLIs.
 *
 * Parity notes (reference = ovhpa/hpnn v0.2):
 *   - scalar type names CHAR/UINT/DOUBLE/BOOL/SHORT/UINT64 mirror
 *     include/libhpnn/common.h:147-160 of the reference so that host code
 *     written against the reference header compiles unchanged;
 *   - `cudastreams` keeps the reference field names (common.h:587-605) but
 *     holds HIP streams; there is no cuBLAS handle (no BLAS anywhere);
 *   - `cudas_mem` keeps the four memory-model names (common.h:580-585).
 *     On MI355X every multi-GPU model is served by RCCL over xGMI; the enum
 *     only reports what the runtime selected.
 */
#ifndef LIBHPNN_COMMON_H
#define LIBHPNN_COMMON_H

#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef char CHAR;
typedef unsigned int UINT;
typedef uint64_t UINT64;
typedef double DOUBLE;
typedef float FLOAT;
typedef short SHORT;
typedef int BOOL;
#ifndef TRUE
#define TRUE 1
#endif
#ifndef FALSE
#define FALSE 0
#endif

/* softmax / cross-entropy regulariser (reference common.h:79) */
#define HPNN_TINY 1e-14

/* opaque HIP stream handle: identical to the HIP runtime typedef */
#ifndef HIP_INCLUDE_HIP_HIP_RUNTIME_API_H
typedef struct ihipStream_t *hipStream_t;
#endif

typedef enum {
    CUDA_MEM_NONE = 0, /* single GPU (or none)                          */
    CUDA_MEM_EXP = 1,  /* replica per GPU, explicit collectives (RCCL)   */
    CUDA_MEM_P2P = 2,  /* peer access enabled between all GPUs           */
    CUDA_MEM_CMM = 3,  /* managed memory (kept for API parity)           */
} cudas_mem;

typedef struct {
    UINT n_gpu;               /* GPUs driven by this process              */
    UINT cuda_n_streams;      /* compute streams per GPU                  */
    hipStream_t *cuda_streams;/* n_gpu*cuda_n_streams, GPU = idx/n_streams */
    cudas_mem mem_model;      /* selected multi-GPU memory model          */
} cudastreams;

/* rank used to gate output: RANK env of a torch.distributed / launcher job */
int hpnn_output_rank(void);

/* rank-0 output helper, reference common.h:81-91 semantic */
#define _OUT(_file, ...)                                                   \
    do {                                                                   \
        if (hpnn_output_rank() == 0) fprintf((_file), __VA_ARGS__);        \
    } while (0)

#ifdef __cplusplus
}
#endif
#endif /* LIBHPNN_COMMON_H */
