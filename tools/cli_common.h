/*
 * Shared option parsing for train_nn / run_nn.
 *
 * Reference flags (tests/train_nn.c:33-58, tests/run_nn.c:39-65):
 *   -h help, -v verbose (repeatable, combinable: -vvv), -x dry run
 *   (train_nn only), -O N host threads, -B N BLAS threads (accepted, no
 *   BLAS here), -S N streams per GPU.  Numeric flags take "-O4" or "-O 4".
 * Extensions: -G N GPUs, -b N minibatch (implies batched mode), -e N epochs,
 *   -m online|batched, -d f64|f32|bf16, -c force the CPU engine,
 *   -l LR learning rate, -a ALPHA momentum,
 *   -r FILE exact-resume state (loaded when present, written after training),
 *   -M FILE JSON-lines metrics (same as HPNN_METRICS=FILE),
 *   -T trace ranges + timing table (same as HPNN_TRACE=1).
 */
#ifndef HPNN_CLI_COMMON_H
#define HPNN_CLI_COMMON_H
#include <libhpnn.h>
#include <libhpnn/observe.h>
#include <ctype.h>
#include <string.h>
#include <stdlib.h>

typedef struct {
    const char *conf;
    int dry;
    UINT threads, blas, streams, gpus, batch, epochs;
    int mode;  /* -1 = from conf */
    int dtype; /* -1 = from conf */
    int force_cpu;
    double lr, alpha;
    const char *state;   /* -r */
    const char *metrics; /* -M */
    int help;
} cli_opts;

/* returns 0 on success, -1 on a syntax error */
static int cli_parse(int argc, char **argv, cli_opts *o, int allow_x) {
    memset(o, 0, sizeof(*o));
    o->conf = "./nn.conf";
    o->mode = -1;
    o->dtype = -1;
    o->lr = -1.0;
    o->alpha = -1.0;
    for (int i = 1; i < argc; i++) {
        const char *a = argv[i];
        if (a[0] != '-' || a[1] == 0) {
            o->conf = a;
            continue;
        }
        for (int j = 1; a[j];) {
            char c = a[j];
            if (c == 'h') {
                o->help = 1;
                return 0;
            }
            if (c == 'v') {
                _NN(inc, verbose)();
                j++;
                continue;
            }
            if (c == 'x' && allow_x) {
                o->dry = 1;
                j++;
                continue;
            }
            if (c == 'c') {
                o->force_cpu = 1;
                j++;
                continue;
            }
            if (c == 'T') {
                hpnn_trace_enable(1);
                j++;
                continue;
            }
            if (strchr("OBSGbemdlarM", c)) {
                const char *val = a[j + 1] ? &a[j + 1] : (i + 1 < argc ? argv[++i] : NULL);
                if (!val) {
                    _OUT(stderr, "syntax error: missing -%c parameter!\n", c);
                    return -1;
                }
                if (strchr("OBSGbe", c)) {
                    if (!isdigit((unsigned char)*val) || atoi(val) <= 0) {
                        _OUT(stderr, "syntax error: bad -%c parameter!\n", c);
                        return -1;
                    }
                    UINT v = (UINT)atoi(val);
                    switch (c) {
                        case 'O': o->threads = v; break;
                        case 'B': o->blas = v; break;
                        case 'S': o->streams = v; break;
                        case 'G': o->gpus = v; break;
                        case 'b': o->batch = v; o->mode = NN_MODE_BATCHED; break;
                        case 'e': o->epochs = v; break;
                    }
                } else if (c == 'm') {
                    o->mode = (val[0] == 'b' || val[0] == 'B') ? NN_MODE_BATCHED : NN_MODE_ONLINE;
                } else if (c == 'd') {
                    o->dtype = !strcmp(val, "bf16") ? NN_DTYPE_BF16 : (!strcmp(val, "f32") ? NN_DTYPE_F32 : NN_DTYPE_F64);
                } else if (c == 'l') {
                    o->lr = atof(val);
                } else if (c == 'a') {
                    o->alpha = atof(val);
                } else if (c == 'r') {
                    o->state = val;
                } else if (c == 'M') {
                    o->metrics = val;
                }
                break; /* a value consumes the rest of the argument */
            }
            _OUT(stderr, "syntax error: unknown option -%c\n", c);
            return -1;
        }
    }
    return 0;
}

static void cli_apply_runtime(const cli_opts *o) {
    if (o->threads) _NN(set, omp_threads)(o->threads);
    if (o->blas) _NN(set, omp_blas)(o->blas);
    if (o->gpus) _NN(set, n_gpu)(o->gpus);
    _NN(set, cuda_streams)(o->streams ? o->streams : 1);
    if (o->dry) _NN(toggle, dry)();
    if (o->metrics) hpnn_metrics_open(o->metrics);
}

static void cli_apply_conf(const cli_opts *o, nn_def *conf) {
    if (o->mode >= 0) _NN(set, mode)(conf, (nn_mode)o->mode);
    if (o->dtype >= 0) _NN(set, dtype)(conf, (nn_dtype)o->dtype);
    if (o->batch) _NN(set, batch)(conf, o->batch);
    if (o->epochs) _NN(set, epochs)(conf, o->epochs);
    if (o->force_cpu) _NN(set, device)(conf, NN_DEVICE_CPU);
    if (o->lr > 0) _NN(set, learning_rate)(conf, o->lr);
    if (o->alpha >= 0) _NN(set, momentum)(conf, o->alpha);
}
#endif
