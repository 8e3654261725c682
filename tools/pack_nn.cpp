/*
 * pack_nn -- pack a directory of libhpnn sample files into one binary file.
 *
 *   pack_nn [-v] <sample_dir> <out_file>
 *
 * train_nn / run_nn accept the pack file wherever a [sample_dir] / [test_dir] is
 * expected (csrc/core/dataset.cpp): no per-file text parsing at training time.  The
 * reference has no equivalent (it parses one text file per sample inside the training
 * loop, libhpnn.c:1236-1242).
 */
#include <libhpnn.h>
#include <string.h>

int main(int argc, char *argv[]) {
    _NN(init, all)(0);
    const char *args[2] = {NULL, NULL};
    int na = 0;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-v")) {
            _NN(inc, verbose)();
            _NN(inc, verbose)();
        } else if (!strcmp(argv[i], "-h") || na == 2) {
            na = -1;
            break;
        } else {
            args[na++] = argv[i];
        }
    }
    if (na != 2) {
        _OUT(stderr, "usage: pack_nn [-v] <sample_dir> <out_file>\n");
        _NN(deinit, all)();
        return -1;
    }
    const BOOL ok = _NN(pack, samples)(args[0], args[1]);
    if (!ok) _OUT(stderr, "packing %s FAILED!\n", args[0]);
    _NN(deinit, all)();
    return ok ? 0 : 1;
}
