/*
 * libhpnn (MI355X-native) -- model definition shared by every engine.
 *
 * A network is a stack of bias-free dense layers, one weight row per neuron
 * (row-major N x M, reference include/libhpnn/ann.h:35-55).  The host copy
 * is FP64 and is the master copy for the CPU engine and for I/O; the GPU
 * engines keep their own device state behind `gpu` (see gpu/engine.h).
 */
#ifndef LIBHPNN_ANN_H
#define LIBHPNN_ANN_H
#include <libhpnn.h>

#ifdef __cplusplus
extern "C" {
#endif

#define _2D_IDX(len, j, i) ((size_t)(len) * (size_t)(j) + (size_t)(i))

typedef struct {
    UINT n_neurons; /* N: rows of W, outputs of the layer  */
    UINT n_inputs;  /* M: cols of W, inputs of the layer   */
    DOUBLE *weights;/* N*M row-major                       */
    DOUBLE *vec;    /* N outputs of the last forward pass  */
} layer_ann;

typedef struct {
    CHAR *name;
    UINT n_inputs;
    DOUBLE *in;        /* n_inputs                             */
    UINT n_hiddens;
    layer_ann *hiddens;/* n_hiddens                            */
    UINT n_outputs;
    layer_ann output;
    DOUBLE **dw;       /* momentum, n_hiddens+1 (NULL if none) */
    UINT max_index;    /* max(n_in, n_out, h_i)                */
    DOUBLE *tmp_cpu;   /* scratch, max_index                   */
    void *gpu;         /* device state (hpnn_gpu_model*)        */
} kernel_ann;

/* allocation / I/O (reference ann.c:113-879) */
kernel_ann *ann_kernel_allocate(UINT n_inputs, UINT n_hiddens, const UINT *hiddens,
                                UINT n_outputs);
void ann_kernel_free(kernel_ann *kernel);
kernel_ann *ann_generate(UINT *seed, UINT n_inputs, UINT n_hiddens, UINT n_outputs,
                         const UINT *hiddens);
kernel_ann *ann_load(const CHAR *filename);
void ann_dump(const kernel_ann *kernel, FILE *out, BOOL exact);
BOOL ann_validate_kernel(const kernel_ann *kernel);
UINT64 ann_n_params(const kernel_ann *kernel);

/* math (reference ann.c:883-888) */
DOUBLE ann_act(DOUBLE x);
DOUBLE ann_dact(DOUBLE y);

/* CPU FP64 engine (reference ann.c / snn.c semantics) */
void ann_kernel_run(kernel_ann *kernel);
void snn_kernel_run(kernel_ann *kernel);
void lnn_kernel_run(kernel_ann *kernel);
void hpnn_cpu_forward(kernel_ann *kernel, nn_type type);
DOUBLE hpnn_cpu_error(const kernel_ann *kernel, nn_type type, const DOUBLE *train);
/* one reference training step; returns Ep(before)-Ep(after re-forward) */
DOUBLE hpnn_cpu_train_step(kernel_ann *kernel, nn_type type, const DOUBLE *train, DOUBLE lr,
                           BOOL momentum, DOUBLE alpha);
BOOL ann_momentum_init(kernel_ann *kernel);
void ann_raz_momentum(kernel_ann *kernel);
void ann_momentum_free(kernel_ann *kernel);

/* per-sample convergence driver (reference ann.c:2281-2467, snn.c:1417-1595)
 * returns the last dEp; *n_iter and *ok report the loop outcome */
DOUBLE hpnn_cpu_train_sample(kernel_ann *kernel, nn_type type, nn_train train,
                             const DOUBLE *in, const DOUBLE *out, DOUBLE lr, DOUBLE alpha,
                             DOUBLE delta, UINT *n_iter, BOOL *ok, DOUBLE *init_err,
                             BOOL *first_ok);

/* reference-compatible entry points */
DOUBLE ann_train_BP(kernel_ann *kernel, DOUBLE *train_in, DOUBLE *train_out, DOUBLE delta);
DOUBLE ann_train_BPM(kernel_ann *kernel, DOUBLE *train_in, DOUBLE *train_out, DOUBLE alpha,
                     DOUBLE delta);
DOUBLE snn_train_BP(kernel_ann *kernel, DOUBLE *train_in, DOUBLE *train_out, DOUBLE delta);
DOUBLE snn_train_BPM(kernel_ann *kernel, DOUBLE *train_in, DOUBLE *train_out, DOUBLE alpha,
                     DOUBLE delta);

#ifdef __cplusplus
}
#endif
#endif /* LIBHPNN_ANN_H */
