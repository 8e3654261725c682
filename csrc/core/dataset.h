/*
 * libhpnn sample sources (internal): a directory of reference sample files
 *  or a packed binary file written by nn_pack_samples.
 *
 * The reference parses one text file per training sample, serially, inside the
 * training loop (libhpnn.c:1236-1242).  Batched training here loads the whole set
 * once -- files parsed in parallel by a host thread pool (OpenMP, -O threads) -- and
 * keeps it resident on the GPU (288 GB of HBM per MI355X holds any dataset of this
 * library's scale); a pack file skips the text parsing altogether.
 */
#ifndef HPNN_DATASET_H
#define HPNN_DATASET_H
#include <libhpnn.h>

#include <string>
#include <vector>

#define HPNN_PACK_MAGIC "HPNNPAK1"

struct HpnnSamples {
    bool packed = false;
    std::string dir;                /* directory source                     */
    std::vector<std::string> names; /* file names (sorted) / packed names   */
    UINT n_in = 0, n_out = 0;       /* packed: dims stored in the file      */
    std::vector<DOUBLE> X, T;       /* packed: all records                  */

    /* path: a directory or a pack file */
    bool open(const char *path);
    size_t size() const { return names.size(); }
    /* record i as malloc'd copies (the nn_read_sample contract) */
    bool get(size_t i, DOUBLE **in, DOUBLE **out) const;
    /* records in `order`, n_in / n_out checked; unreadable or mis-sized records are
     * skipped (reference: libhpnn.c:1236-1242); directory files are parsed by
     * `threads` host threads.  Returns the number of records loaded. */
    size_t load(const std::vector<UINT> &order, UINT n_in, UINT n_out, int threads, std::vector<DOUBLE> &Xo,
                std::vector<DOUBLE> &To) const;
};

/* FNV-1a 64-bit checksum (pack and state files) */
UINT64 hpnn_fnv1a(const void *data, size_t n, UINT64 h);
#define HPNN_FNV_SEED 1469598103934665603ULL

#endif
