/*
 * libhpnn runtime layer (MI355X-native).
 *
 * Parity: reference src/libhpnn.c:58-539 (global nn_runtime, capability bits,
 * init/deinit of the OMP/MPI/CUDA/BLAS tiers, thread/GPU/stream setters).
 * Design differences:
 *   - "MPI" is the torch.distributed / launcher world read from the
 *     environment (RANK / WORLD_SIZE / LOCAL_RANK): one process per GPU, no
 *     libmpi.  The collectives live in csrc/dist (RCCL over xGMI).
 *   - "CUDA" is HIP on gfx950.  Streams are created per GPU on demand, so a
 *     caller that forgets nn_set_cuda_streams (reference quirk,
 *     libhpnn.c:169-170) still gets one stream per GPU.
 *   - the memory-model probe checks every GPU pair for peer access (the
 *     reference probed GPU0 against itself, libhpnn.c:251-256).
 *   - there is no BLAS tier: nn_init_BLAS succeeds and only records -B.
 */
#include <libhpnn.h>
#include <libhpnn/observe.h>
#include <libhpnn/devmem.h>
#include <hip/hip_runtime_api.h>
#include <omp.h>
#include <stdarg.h>
#include <string.h>

#include "runtime_internal.h"

static nn_runtime lib_runtime;
static BOOL runtime_ready = FALSE;
static int g_device_base = 0;   /* first HIP device owned by this process */
static int g_output_rank = -1;

extern "C" int hpnn_output_rank(void) {
    if (g_output_rank < 0) {
        const char *r = getenv("RANK");
        g_output_rank = r ? atoi(r) : 0;
    }
    return g_output_rank;
}

static int env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    return v ? atoi(v) : dflt;
}

int hpnn_rt_device(UINT gpu) { return g_device_base + (int)gpu; }

hipStream_t hpnn_rt_stream(UINT gpu, UINT idx) {
    cudastreams *c = &lib_runtime.cudas;
    if (c->n_gpu == 0) return NULL;
    if (c->cuda_streams == NULL) _NN(set, cuda_streams)(c->cuda_n_streams ? c->cuda_n_streams : 1);
    if (c->cuda_streams == NULL) return NULL;
    UINT ns = c->cuda_n_streams;
    return c->cuda_streams[gpu * ns + (idx % ns)];
}

BOOL hpnn_rt_gpu_available(void) {
    return (lib_runtime.capability & NN_CAP_CUDA) && lib_runtime.cudas.n_gpu > 0;
}

static void nn_init_runtime(void) {
    memset(&lib_runtime, 0, sizeof(lib_runtime));
    lib_runtime.capability = (nn_cap)(NN_CAP_OMP | NN_CAP_MPI);
    lib_runtime.nn_verbose = 0;
    lib_runtime.nn_dry = FALSE;
    lib_runtime.nn_num_threads = 1;
    lib_runtime.nn_num_blas = 1;
    lib_runtime.nn_num_tasks = 1;
    lib_runtime.cudas.n_gpu = 0;
    lib_runtime.cudas.cuda_n_streams = 1;
    lib_runtime.cudas.cuda_streams = NULL;
    lib_runtime.cudas.mem_model = CUDA_MEM_NONE;
    runtime_ready = TRUE;
}

static void ensure_runtime(void) {
    if (!runtime_ready) nn_init_runtime();
}

/* ---------------- verbosity ---------------- */
extern "C" void _NN(inc, verbose)(void) { ensure_runtime(); lib_runtime.nn_verbose++; }
extern "C" void _NN(dec, verbose)(void) {
    ensure_runtime();
    if (lib_runtime.nn_verbose > 0) lib_runtime.nn_verbose--;
}
extern "C" void _NN(set, verbose)(SHORT v) { ensure_runtime(); lib_runtime.nn_verbose = v; }
extern "C" void _NN(get, verbose)(SHORT *v) { ensure_runtime(); *v = lib_runtime.nn_verbose; }
extern "C" SHORT _NN(return, verbose)(void) { ensure_runtime(); return lib_runtime.nn_verbose; }
/* the reference XORs the flag with itself (always FALSE, libhpnn.c:88-90);
 * here -x really toggles "dry run": train_nn then skips the kernel dumps */
extern "C" void _NN(toggle, dry)(void) { ensure_runtime(); lib_runtime.nn_dry = !lib_runtime.nn_dry; }
extern "C" BOOL _NN(return, dry)(void) { ensure_runtime(); return lib_runtime.nn_dry; }

/* ---------------- capabilities ---------------- */
extern "C" void _NN(get, capabilities)(nn_cap *cap) { ensure_runtime(); *cap = lib_runtime.capability; }
extern "C" void _NN(unset, capability)(nn_cap cap) {
    ensure_runtime();
    lib_runtime.capability = (nn_cap)(lib_runtime.capability & ~cap);
}
extern "C" nn_cap _NN(return, capabilities)(void) { ensure_runtime(); return lib_runtime.capability; }

/* ---------------- tiers ---------------- */
extern "C" BOOL _NN(init, OMP)(void) {
    ensure_runtime();
    lib_runtime.nn_num_threads = 1;
    return TRUE;
}

extern "C" BOOL _NN(init, MPI)(void) {
    ensure_runtime();
    int ws = env_int("WORLD_SIZE", 1);
    lib_runtime.nn_num_tasks = ws > 0 ? (UINT)ws : 1;
    if (lib_runtime.nn_num_tasks < 2)
        NN_DBG(stdout, "single process run (WORLD_SIZE<2).\n");
    return TRUE;
}

extern "C" BOOL _NN(init, CUDA)(void) {
    ensure_runtime();
    /* HPNN_DEBUG=1: serialise and check every HIP launch / copy (takes effect when the
     * HIP runtime starts here, i.e. before any other HIP call of the process) */
    if (hpnn_debug_enabled()) {
        setenv("AMD_SERIALIZE_KERNEL", "3", 0);
        setenv("AMD_SERIALIZE_COPY", "3", 0);
        NN_WARN(stdout, "debug mode: serialised HIP launches and copies.\n");
    }
    int n = 0;
    const char *force_cpu = getenv("HPNN_FORCE_CPU");
    if (force_cpu && force_cpu[0] == '1') n = 0;
    else if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    if (n < 1) {
        lib_runtime.capability = (nn_cap)(lib_runtime.capability & ~(NN_CAP_CUDA | NN_CAP_RCCL | NN_CAP_MFMA));
        lib_runtime.cudas.n_gpu = 0;
        NN_WARN(stdout, "no GPU found, CPU engine only.\n");
        return FALSE;
    }
    /* one process per GPU under a launcher: own device LOCAL_RANK only */
    int ws = env_int("WORLD_SIZE", 1);
    int lr = env_int("LOCAL_RANK", -1);
    if (ws > 1 && lr >= 0 && lr < n) {
        g_device_base = lr;
        lib_runtime.cudas.n_gpu = 1;
    } else {
        g_device_base = 0;
        lib_runtime.cudas.n_gpu = (UINT)n;
    }
    lib_runtime.capability = (nn_cap)(lib_runtime.capability | NN_CAP_CUDA | NN_CAP_RCCL | NN_CAP_MFMA);
    NN_WARN(stdout, "HIP started, using %u GPU(s).\n", lib_runtime.cudas.n_gpu);
    hpnn_rt_probe_memory_model();
    return TRUE;
}

void hpnn_rt_probe_memory_model(void) {
    cudastreams *c = &lib_runtime.cudas;
    c->mem_model = CUDA_MEM_NONE;
    if (c->n_gpu < 2) return;
    BOOL all = TRUE;
    for (UINT a = 0; a < c->n_gpu; a++)
        for (UINT b = 0; b < c->n_gpu; b++) {
            if (a == b) continue;
            int ok = 0;
            hipDeviceCanAccessPeer(&ok, hpnn_rt_device(a), hpnn_rt_device(b));
            all = all && ok;
        }
    if (all) {
        for (UINT a = 0; a < c->n_gpu; a++) {
            hipSetDevice(hpnn_rt_device(a));
            for (UINT b = 0; b < c->n_gpu; b++)
                if (a != b) {
                    hipError_t e = hipDeviceEnablePeerAccess(hpnn_rt_device(b), 0);
                    if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
                }
        }
        c->mem_model = CUDA_MEM_P2P;
    } else {
        /* the reference's fallback order (libhpnn.c:245-280): peer access, then managed
         * memory with concurrent access on every device, then explicit copies.  The engines
         * treat CMM like EXP (a replica per device, explicit collectives): on an xGMI node
         * every pair has peer access, so CMM is only reached on a partial topology. */
        BOOL cmm = TRUE;
        for (UINT a = 0; a < c->n_gpu; a++) {
            int mm = 0, conc = 0;
            hipDeviceGetAttribute(&mm, hipDeviceAttributeManagedMemory, hpnn_rt_device(a));
            hipDeviceGetAttribute(&conc, hipDeviceAttributeConcurrentManagedAccess, hpnn_rt_device(a));
            cmm = cmm && mm && conc;
        }
        c->mem_model = cmm ? CUDA_MEM_CMM : CUDA_MEM_EXP;
    }
    switch (c->mem_model) {
    case CUDA_MEM_P2P: NN_DBG(stdout, "multi-GPU will use peer access between all GPUs\n"); break;
    case CUDA_MEM_CMM: NN_DBG(stdout, "multi-GPU will use managed memory (explicit collectives)\n"); break;
    case CUDA_MEM_EXP: NN_DBG(stdout, "multi-GPU using explicit collectives\n"); break;
    default: break;
    }
    hipSetDevice(hpnn_rt_device(0));
}

extern "C" BOOL _NN(init, BLAS)(void) {
    ensure_runtime();
    lib_runtime.nn_num_blas = 1;
    return TRUE;
}

extern "C" int _NN(init, all)(UINT init_verbose) {
    nn_init_runtime();
    lib_runtime.nn_verbose = (SHORT)init_verbose;
    _NN(init, MPI)();
    _NN(init, OMP)();
    _NN(init, CUDA)();
    _NN(init, BLAS)();
    lib_runtime.nn_verbose = 0;
    return 0;
}

static void destroy_streams(void) {
    cudastreams *c = &lib_runtime.cudas;
    if (c->cuda_streams == NULL) return;
    for (UINT g = 0; g < c->n_gpu; g++) {
        hipSetDevice(hpnn_rt_device(g));
        for (UINT s = 0; s < c->cuda_n_streams; s++) {
            hipStream_t st = c->cuda_streams[g * c->cuda_n_streams + s];
            if (st) hipStreamDestroy(st);
        }
    }
    free(c->cuda_streams);
    c->cuda_streams = NULL;
}

extern "C" BOOL _NN(deinit, OMP)(void) { return TRUE; }
extern "C" BOOL _NN(deinit, MPI)(void) { return TRUE; }
extern "C" BOOL _NN(deinit, CUDA)(void) {
    ensure_runtime();
    if (!(lib_runtime.capability & NN_CAP_CUDA)) return TRUE;
    hpnn_rt_release_device_state();
    hpnn_dev_trim(); /* cached device blocks back to the driver */
    destroy_streams();
    return TRUE;
}
extern "C" BOOL _NN(deinit, BLAS)(void) { return TRUE; }
extern "C" int _NN(deinit, all)(void) {
    _NN(deinit, CUDA)();
    _NN(deinit, BLAS)();
    _NN(deinit, OMP)();
    _NN(deinit, MPI)();
    runtime_ready = FALSE;
    return 0;
}

/* ---------------- parameters ---------------- */
extern "C" BOOL _NN(set, omp_threads)(UINT n) {
    ensure_runtime();
    if (n == 0) return FALSE;
    lib_runtime.nn_num_threads = n;
    omp_set_num_threads((int)n);
    return TRUE;
}
extern "C" BOOL _NN(get, omp_threads)(UINT *n) { ensure_runtime(); *n = lib_runtime.nn_num_threads; return TRUE; }
extern "C" int _NN(return, omp_threads)(void) { ensure_runtime(); return (int)lib_runtime.nn_num_threads; }
extern "C" BOOL _NN(set, mpi_tasks)(UINT n) {
    ensure_runtime();
    if (n == 0) return FALSE;
    lib_runtime.nn_num_tasks = n;
    return TRUE;
}
extern "C" BOOL _NN(get, mpi_tasks)(UINT *n) { ensure_runtime(); *n = lib_runtime.nn_num_tasks; return TRUE; }
extern "C" BOOL _NN(get, curr_mpi_task)(UINT *t) { *t = (UINT)hpnn_output_rank(); return TRUE; }
extern "C" BOOL _NN(set, n_gpu)(UINT n) {
    ensure_runtime();
    int avail = 0;
    if (hipGetDeviceCount(&avail) != hipSuccess) avail = 0;
    if (n == 0 || (int)(n + g_device_base) > avail) return FALSE;
    destroy_streams();
    lib_runtime.cudas.n_gpu = n;
    hpnn_rt_probe_memory_model();
    return TRUE;
}
extern "C" BOOL _NN(get, n_gpu)(UINT *n) { ensure_runtime(); *n = lib_runtime.cudas.n_gpu; return TRUE; }
extern "C" BOOL _NN(set, cuda_streams)(UINT n) {
    ensure_runtime();
    if (n == 0) return FALSE;
    cudastreams *c = &lib_runtime.cudas;
    destroy_streams();
    c->cuda_n_streams = n;
    if (c->n_gpu == 0) return TRUE; /* nothing to create on a CPU-only box */
    c->cuda_streams = (hipStream_t *)calloc((size_t)c->n_gpu * n, sizeof(hipStream_t));
    for (UINT g = 0; g < c->n_gpu; g++) {
        hipSetDevice(hpnn_rt_device(g));
        for (UINT s = 0; s < n; s++) {
            if (hipStreamCreateWithFlags(&c->cuda_streams[g * n + s], hipStreamNonBlocking) != hipSuccess) {
                NN_ERROR(stderr, "HIP: can't create stream %u on GPU[%u]\n", s, g);
                return FALSE;
            }
        }
    }
    hipSetDevice(hpnn_rt_device(0));
    return TRUE;
}
extern "C" BOOL _NN(get, cuda_streams)(UINT *n) { ensure_runtime(); *n = lib_runtime.cudas.cuda_n_streams; return TRUE; }
extern "C" BOOL _NN(set, omp_blas)(UINT n) {
    ensure_runtime();
    if (n == 0) return FALSE;
    lib_runtime.nn_num_blas = n;
    return TRUE;
}
extern "C" BOOL _NN(get, omp_blas)(UINT *n) { ensure_runtime(); *n = lib_runtime.nn_num_blas; return TRUE; }
extern "C" cudastreams *_NN(return, cudas)(void) { ensure_runtime(); return &lib_runtime.cudas; }

nn_runtime *hpnn_rt_get(void) { ensure_runtime(); return &lib_runtime; }

extern "C" const char *_NN(return, version)(void) { return "libhpnn-mi355x 0.3.0 (gfx950)"; }
