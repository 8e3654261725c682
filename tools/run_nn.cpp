/*
 * run_nn -- evaluate a libhpnn network on the test directory of a conf.
 * Workflow parity with the reference CLI (tests/run_nn.c:66-234): init ->
 * flags -> nn_load_conf -> nn_run_kernel (prints [PASS]/[FAIL idx=]) ->
 * deinit.  Prints a final accuracy line at verbosity >= 1.
 */
#include <libhpnn.h>
#include "cli_common.h"

static void dump_help(void) {
    _OUT(stdout, "****************************************\n");
    _OUT(stdout, " usage: run_nn [-options] [input]       \n");
    _OUT(stdout, "****************************************\n");
    _OUT(stdout, "options:                               *\n");
    _OUT(stdout, "-h \tdisplay this help;                *\n");
    _OUT(stdout, "-v \tincrease verbosity;               *\n");
    _OUT(stdout, "-O N\thost threads.                     *\n");
    _OUT(stdout, "-B N\tBLAS threads (accepted, unused).  *\n");
    _OUT(stdout, "-S N\tHIP streams per GPU.              *\n");
    _OUT(stdout, "-G N\tnumber of GPUs.                   *\n");
    _OUT(stdout, "-c \tforce the CPU engine.              *\n");
    _OUT(stdout, "****************************************\n");
    _OUT(stdout, "input: neural network conf file        *\n");
    _OUT(stdout, "(default ./nn.conf)                    *\n");
    _OUT(stdout, "****************************************\n");
}

int main(int argc, char *argv[]) {
    cli_opts o;
    _NN(init, all)(0);
    if (cli_parse(argc, argv, &o, 0)) {
        dump_help();
        _NN(deinit, all)();
        return -1;
    }
    if (o.help) {
        dump_help();
        _NN(deinit, all)();
        return 0;
    }
    cli_apply_runtime(&o);
    nn_def *neural = _NN(load, conf)(o.conf);
    if (!neural) {
        _OUT(stderr, "FAILED to read NN configuration file! (ABORTING)\n");
        _NN(deinit, all)();
        return -1;
    }
    cli_apply_conf(&o, neural);
    _NN(run, kernel)(neural);
    if (_NN(return, verbose)() > 0)
        _OUT(stdout, "ACCURACY: %u/%u\n", _NN(return, last_pass)(), _NN(return, last_total)());
    _NN(deinit, conf)(neural);
    free(neural);
    _NN(deinit, all)();
    return 0;
}
