/*
 * libhpnn -- MI355X-native feed-forward neural network library.
 *
 * Public C API.  Every symbol, enum value and struct name of the reference
 * header (ovhpa/hpnn include/libhpnn.h:26-215) is provided with the same
 * meaning, so a program written against libhpnn links against this library
 * unchanged.  Extensions (batched training, precision selection, learning
 * rate / momentum / epoch control, GPU selection) are appended after the
 * reference surface and never change the reference semantics.
 */
#ifndef LIBHPNN_H
#define LIBHPNN_H
#include <libhpnn/common.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- capabilities (reference libhpnn.h:26-35) ---- */
typedef enum {
    NN_CAP_NONE = 0,
    NN_CAP_OMP = (1 << 0),    /* host thread pool                          */
    NN_CAP_MPI = (1 << 1),    /* multi-process (torch.distributed / RCCL)  */
    NN_CAP_CUDA = (1 << 2),   /* GPU (HIP on MI355X)                        */
    NN_CAP_CUBLAS = (1 << 3), /* never set: no vendor BLAS is used          */
    /* (1<<4) reserved (OCL in the reference) */
    NN_CAP_PBLAS = (1 << 5),  /* never set                                  */
    NN_CAP_SBLAS = (1 << 6),  /* never set                                  */
    NN_CAP_RCCL = (1 << 7),   /* extension: RCCL collectives available      */
    NN_CAP_MFMA = (1 << 8),   /* extension: gfx950 MFMA kernels loaded      */
} nn_cap;

typedef struct {
    nn_cap capability;
    SHORT nn_verbose;
    BOOL nn_dry;
    UINT nn_num_threads;
    UINT nn_num_blas;
    UINT nn_num_tasks;
    cudastreams cudas;
} nn_runtime;

/* ---- network / training types (reference libhpnn.h:51-66) ---- */
typedef enum {
    NN_TYPE_ANN = 0, /* bipolar sigmoid on every layer, MSE               */
    NN_TYPE_LNN = 1, /* sigmoid hidden + linear output (extension: works) */
    NN_TYPE_SNN = 2, /* sigmoid hidden + softmax output, cross-entropy    */
    NN_TYPE_UKN = -1,
} nn_type;

typedef enum {
    NN_TRAIN_BP = 0,
    NN_TRAIN_BPM = 1,
    NN_TRAIN_CG = 2,   /* parsed, not implemented (as in the reference)  */
    NN_TRAIN_SPLX = 3, /* parsed, not implemented (as in the reference)  */
    NN_TRAIN_UKN = -1,
} nn_train;

/* reference hyper-parameters (libhpnn.h:67-74) */
#define BP_LEARN_RATE 0.001
#define MIN_BP_ITER 31
#define MAX_BP_ITER 102399
#define DELTA_BP 1E-6
#define BPM_LEARN_RATE 0.0005
#define MIN_BPM_ITER 15
#define MAX_BPM_ITER 102399
#define DELTA_BPM 1E-6
/* learning rate used by every GPU path and the CPU SNN path of the
 * reference (cuda_ann.cu:2094, cuda_snn.cu:1918, snn.c:799) */
#define GPU_LEARN_RATE 0.01
#define BPM_MOMENTUM 0.2

/* ---- extensions: execution mode and precision ---- */
typedef enum {
    NN_MODE_ONLINE = 0,  /* reference semantics: batch 1, per-sample loop */
    NN_MODE_BATCHED = 1, /* minibatch SGD / momentum, one pass per sample */
} nn_mode;

typedef enum {
    NN_DTYPE_F64 = 0,  /* FP64 everywhere (reference precision)          */
    NN_DTYPE_F32 = 1,  /* FP32 compute                                   */
    NN_DTYPE_BF16 = 2, /* BF16 MFMA, FP32 accumulate + FP32 master       */
} nn_dtype;

typedef enum {
    NN_DEVICE_AUTO = 0, /* GPU when present, else CPU                     */
    NN_DEVICE_CPU = 1,
    NN_DEVICE_GPU = 2,
} nn_device;

typedef enum {
    NN_PARALLEL_DP = 0,
    NN_PARALLEL_TP = 1,
} nn_parallel;

typedef struct {
    nn_runtime *rr;  /* link to the runtime parameters */
    CHAR *name;
    nn_type type;
    BOOL need_init;
    UINT seed;
    void *kernel;    /* kernel_ann* */
    CHAR *f_kernel;
    nn_train train;
    CHAR *samples;
    CHAR *tests;
    /* -- extensions (optional conf keys, see docs/FORMATS.md) -- */
    nn_mode mode;
    nn_dtype dtype;
    nn_device device;
    UINT batch;      /* minibatch size in batched mode (default 256) */
    UINT epochs;     /* passes over the sample directory (default 1) */
    DOUBLE lr;       /* <=0: reference default for the path          */
    DOUBLE momentum; /* <0 : reference default 0.2                   */
    /* -- training progress (exact resume, nn_dump_state / nn_load_state) -- */
    UINT epochs_done;    /* batched epochs completed on this kernel       */
    UINT64 samples_seen; /* training samples processed on this kernel     */
    BOOL resume;         /* start batched training from the saved momentum */
    /* -- batched multi-GPU layout: [parallel] dp (replicas) | tp (rows of every hidden
     *    layer sharded over the GPUs / ranks; [dtype] f64 or f32) -- */
    nn_parallel parallel;
} nn_def;

#define _NN(a, b) nn_##a##_##b

/* logging (reference libhpnn.h:95-122) */
#define NN_DBG(_file, ...)                                                 \
    do {                                                                   \
        if ((_NN(return, verbose)()) > 2) {                                \
            _OUT((_file), "NN(DBG): ");                                   \
            _OUT((_file), __VA_ARGS__);                                    \
        }                                                                  \
    } while (0)
#define NN_OUT(_file, ...)                                                 \
    do {                                                                   \
        if ((_NN(return, verbose)()) > 1) {                                \
            _OUT((_file), "NN: ");                                        \
            _OUT((_file), __VA_ARGS__);                                    \
        }                                                                  \
    } while (0)
#define NN_COUT(_file, ...)                                                \
    do {                                                                   \
        if ((_NN(return, verbose)()) > 1) { _OUT((_file), __VA_ARGS__); }  \
    } while (0)
#define NN_WARN(_file, ...)                                                \
    do {                                                                   \
        if ((_NN(return, verbose)()) > 0) {                                \
            _OUT((_file), "NN(WARN): ");                                  \
            _OUT((_file), __VA_ARGS__);                                    \
        }                                                                  \
    } while (0)
#define NN_ERROR(_file, ...)                                               \
    do {                                                                   \
        _OUT((_file), "NN(ERR): ");                                       \
        _OUT((_file), __VA_ARGS__);                                        \
    } while (0)
#define NN_WRITE _OUT

/* ---- library init / runtime ---- */
void _NN(inc, verbose)(void);
void _NN(dec, verbose)(void);
void _NN(set, verbose)(SHORT verbosity);
void _NN(get, verbose)(SHORT *verbosity);
SHORT _NN(return, verbose)(void);
void _NN(toggle, dry)(void);
BOOL _NN(return, dry)(void);
void _NN(get, capabilities)(nn_cap *capabilities);
void _NN(unset, capability)(nn_cap capability);
nn_cap _NN(return, capabilities)(void);
BOOL _NN(init, OMP)(void);
BOOL _NN(init, MPI)(void);
BOOL _NN(init, CUDA)(void);
BOOL _NN(init, BLAS)(void);
int _NN(init, all)(UINT init_verbose);
BOOL _NN(deinit, OMP)(void);
BOOL _NN(deinit, MPI)(void);
BOOL _NN(deinit, CUDA)(void);
BOOL _NN(deinit, BLAS)(void);
int _NN(deinit, all)(void);

BOOL _NN(set, omp_threads)(UINT n_threads);
BOOL _NN(get, omp_threads)(UINT *n_threads);
int _NN(return, omp_threads)(void);
BOOL _NN(set, mpi_tasks)(UINT n_tasks);
BOOL _NN(get, mpi_tasks)(UINT *n_tasks);
BOOL _NN(get, curr_mpi_task)(UINT *task);
BOOL _NN(set, n_gpu)(UINT n_gpu);
BOOL _NN(get, n_gpu)(UINT *n_gpu);
BOOL _NN(set, cuda_streams)(UINT n_streams);
BOOL _NN(get, cuda_streams)(UINT *n_streams);
BOOL _NN(set, omp_blas)(UINT n_blas);
BOOL _NN(get, omp_blas)(UINT *n_blas);
cudastreams *_NN(return, cudas)(void);

/* ---- configuration ---- */
void _NN(init, conf)(nn_def *conf);
void _NN(deinit, conf)(nn_def *conf);
void _NN(set, name)(nn_def *conf, const CHAR *name);
void _NN(get, name)(nn_def *conf, CHAR **name);
char *_NN(return, name)(nn_def *conf);
void _NN(set, type)(nn_def *conf, nn_type type);
void _NN(get, type)(nn_def *conf, nn_type *type);
nn_type _NN(return, type)(nn_def *conf);
void _NN(set, need_init)(nn_def *conf, BOOL need_init);
void _NN(get, need_init)(nn_def *conf, BOOL *need_init);
BOOL _NN(return, need_init)(nn_def *conf);
void _NN(set, seed)(nn_def *conf, UINT seed);
void _NN(get, seed)(nn_def *conf, UINT *seed);
UINT _NN(return, seed)(nn_def *conf);
void _NN(set, kernel_filename)(nn_def *conf, CHAR *f_kernel);
void _NN(get, kernel_filename)(nn_def *conf, CHAR **f_kernel);
char *_NN(return, kernel_filename)(nn_def *conf);
void _NN(set, train)(nn_def *conf, nn_train train);
void _NN(get, train)(nn_def *conf, nn_train *train);
nn_train _NN(return, train)(nn_def *conf);
void _NN(set, samples_directory)(nn_def *conf, CHAR *samples);
void _NN(get, samples_directory)(nn_def *conf, CHAR **samples);
char *_NN(return, samples_directory)(nn_def *conf);
void _NN(set, tests_directory)(nn_def *conf, CHAR *tests);
void _NN(get, tests_directory)(nn_def *conf, CHAR **tests);
char *_NN(return, tests_directory)(nn_def *conf);
nn_def *_NN(load, conf)(const CHAR *filename);
void _NN(dump, conf)(nn_def *conf, FILE *fp);

/* ---- kernel (weights) ---- */
void _NN(free, kernel)(nn_def *conf);
BOOL _NN(generate, kernel)(nn_def *conf, ...);
BOOL _NN(load, kernel)(nn_def *conf);
void _NN(dump, kernel)(nn_def *conf, FILE *output);

UINT _NN(get, n_inputs)(nn_def *conf);
UINT _NN(get, n_hiddens)(nn_def *conf);
UINT _NN(get, n_outputs)(nn_def *conf);
UINT _NN(get, h_neurons)(nn_def *conf, UINT layer);

/* ---- samples / execution ---- */
BOOL _NN(read, sample)(CHAR *filename, DOUBLE **in, DOUBLE **out);
BOOL _NN(train, kernel)(nn_def *conf);
void _NN(run, kernel)(nn_def *conf);

/* ---- extensions ---- */
void _NN(set, mode)(nn_def *conf, nn_mode mode);
nn_mode _NN(return, mode)(nn_def *conf);
void _NN(set, dtype)(nn_def *conf, nn_dtype dtype);
nn_dtype _NN(return, dtype)(nn_def *conf);
void _NN(set, device)(nn_def *conf, nn_device device);
nn_device _NN(return, device)(nn_def *conf);
void _NN(set, batch)(nn_def *conf, UINT batch);
UINT _NN(return, batch)(nn_def *conf);
void _NN(set, epochs)(nn_def *conf, UINT epochs);
UINT _NN(return, epochs)(nn_def *conf);
void _NN(set, learning_rate)(nn_def *conf, DOUBLE lr);
DOUBLE _NN(return, learning_rate)(nn_def *conf);
void _NN(set, momentum)(nn_def *conf, DOUBLE alpha);
DOUBLE _NN(return, momentum)(nn_def *conf);
/* write the kernel with %.17g (bit-exact round trip) instead of %17.15f */
void _NN(dump, kernel_exact)(nn_def *conf, FILE *output);
/* number of accurate predictions of the last nn_run_kernel call */
UINT _NN(return, last_pass)(void);
UINT _NN(return, last_total)(void);
/* library version string */
const char *_NN(return, version)(void);
/* exact training state sidecar (bit-exact FP64 weights, momentum, seed, progress,
 * checksum): kernel.opt stays the interchange format, the state file resumes exactly */
BOOL _NN(dump, state)(nn_def *conf, const CHAR *filename);
BOOL _NN(load, state)(nn_def *conf, const CHAR *filename);
UINT _NN(return, epochs_done)(nn_def *conf);
/* pack a directory of sample files into one binary file; train / run accept a pack
 * file wherever a sample or test directory is expected */
BOOL _NN(pack, samples)(const CHAR *dir, const CHAR *filename);
/* the same file from n records in memory (X: n x n_in, T: n x n_out, row-major) */
BOOL _NN(pack, arrays)(const CHAR *filename, const DOUBLE *X, const DOUBLE *T, UINT n, UINT n_in, UINT n_out);

#ifdef __cplusplus
}
#endif
#endif /* LIBHPNN_H */
