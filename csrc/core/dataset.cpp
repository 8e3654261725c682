/*
 * libhpnn sample sources: directory of reference sample files or packed binary file,
 * parallel loading, nn_pack_samples.  See dataset.h.
 *
 * Pack file layout (little endian):
 *   char magic[8] = "HPNNPAK1"
 *   u32 n, n_in, n_out, reserved
 *   u64 names_bytes; names_bytes of NUL-terminated file names (record order)
 *   f64 X[n * n_in]; f64 T[n * n_out]
 *   u64 FNV-1a checksum of X and T
 */
#include "dataset.h"

#include <ctype.h>
#include <dirent.h>
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>

UINT64 hpnn_fnv1a(const void *data, size_t n, UINT64 h) {
    const unsigned char *p = (const unsigned char *)data;
    for (size_t i = 0; i < n; i++) {
        h ^= p[i];
        h *= 1099511628211ULL;
    }
    return h;
}

namespace {

bool slurp(const char *path, std::string &s) {
    FILE *fp = fopen(path, "rb");
    if (!fp) return false;
    char buf[1 << 16];
    size_t r;
    s.clear();
    while ((r = fread(buf, 1, sizeof buf, fp)) > 0) s.append(buf, r);
    fclose(fp);
    return true;
}

/* parse "[tag] N" then N numbers (comments after the count are skipped) */
bool parse_block(const char *text, const char *tag, std::vector<DOUBLE> &v) {
    const char *p = strstr(text, tag);
    if (!p) return false;
    p = strchr(p, ']');
    if (!p) return false;
    char *end;
    const unsigned long n = strtoul(p + 1, &end, 10);
    if (end == p + 1 || n == 0) return false;
    p = strchr(end, '\n');
    if (!p) return false;
    v.resize(n);
    for (unsigned long i = 0; i < n; i++) {
        const double x = strtod(p, &end);
        if (end == p) return false;
        v[i] = x;
        p = end;
    }
    return true;
}

bool read_sized(const std::string &path, std::vector<DOUBLE> &in, std::vector<DOUBLE> &out) {
    std::string s;
    if (!slurp(path.c_str(), s)) return false;
    return parse_block(s.c_str(), "[input", in) && parse_block(s.c_str(), "[output", out);
}

bool is_pack(const char *path) {
    struct stat st;
    if (stat(path, &st) != 0 || !S_ISREG(st.st_mode)) return false;
    FILE *fp = fopen(path, "rb");
    if (!fp) return false;
    char m[8] = {0};
    const bool ok = fread(m, 1, 8, fp) == 8 && !memcmp(m, HPNN_PACK_MAGIC, 8);
    fclose(fp);
    return ok;
}

/* parse every file of `names` (parallel, `threads`), keep the ones with the given
 * dims (0 = any, fixed by the first readable file) */
size_t load_dir(const std::string &dir, const std::vector<std::string> &names, const std::vector<UINT> &order,
                UINT &ni, UINT &no, int threads, std::vector<DOUBLE> &Xo, std::vector<DOUBLE> &To,
                std::vector<std::string> *kept) {
    const long m = (long)order.size();
    std::vector<std::vector<DOUBLE>> xin(m), tout(m);
    std::vector<char> rd(m, 0);
#pragma omp parallel for num_threads(threads > 0 ? threads : 1) schedule(dynamic, 16)
    for (long j = 0; j < m; j++) rd[j] = read_sized(dir + "/" + names[order[j]], xin[j], tout[j]);
    Xo.clear();
    To.clear();
    size_t cnt = 0;
    for (long j = 0; j < m; j++) {
        if (rd[j] && ni == 0 && no == 0) {
            ni = (UINT)xin[j].size();
            no = (UINT)tout[j].size();
        }
        if (!rd[j] || xin[j].size() != ni || tout[j].size() != no) {
            NN_WARN(stderr, "skipping sample %s (unreadable or wrong size)\n", names[order[j]].c_str());
            continue;
        }
        Xo.insert(Xo.end(), xin[j].begin(), xin[j].end());
        To.insert(To.end(), tout[j].begin(), tout[j].end());
        if (kept) kept->push_back(names[order[j]]);
        cnt++;
    }
    return cnt;
}

}  // namespace

bool HpnnSamples::open(const char *path) {
    names.clear();
    X.clear();
    T.clear();
    packed = false;
    if (!path) return false;
    if (is_pack(path)) {
        FILE *fp = fopen(path, "rb");
        if (!fp) return false;
        char m[8];
        UINT hdr[4];
        UINT64 nb = 0, sum = 0;
        bool ok = fread(m, 1, 8, fp) == 8 && fread(hdr, 4, 4, fp) == 4 && fread(&nb, 8, 1, fp) == 1;
        std::string nm;
        if (ok) {
            nm.resize(nb);
            ok = nb == 0 || fread(&nm[0], 1, nb, fp) == nb;
        }
        if (ok) {
            n_in = hdr[1];
            n_out = hdr[2];
            X.resize((size_t)hdr[0] * n_in);
            T.resize((size_t)hdr[0] * n_out);
            ok = fread(X.data(), 8, X.size(), fp) == X.size() && fread(T.data(), 8, T.size(), fp) == T.size() &&
                 fread(&sum, 8, 1, fp) == 1;
        }
        fclose(fp);
        if (ok) {
            UINT64 h = hpnn_fnv1a(X.data(), X.size() * 8, HPNN_FNV_SEED);
            h = hpnn_fnv1a(T.data(), T.size() * 8, h);
            if (h != sum) {
                NN_ERROR(stderr, "pack file %s: checksum mismatch (corrupted)\n", path);
                ok = false;
            }
        }
        if (!ok) {
            NN_ERROR(stderr, "can't read pack file %s\n", path);
            X.clear();
            T.clear();
            return false;
        }
        for (size_t i = 0, s = 0; i < nb && names.size() < hdr[0]; i++)
            if (nm[i] == 0) {
                names.emplace_back(nm.substr(s, i - s));
                s = i + 1;
            }
        while (names.size() < hdr[0]) names.emplace_back("s" + std::to_string(names.size()));
        packed = true;
        return true;
    }
    DIR *d = opendir(path);
    if (!d) return false;
    struct dirent *e;
    while ((e = readdir(d)) != NULL) {
        if (e->d_name[0] == '.') continue;
        names.emplace_back(e->d_name);
    }
    closedir(d);
    std::sort(names.begin(), names.end());
    dir = path;
    return true;
}

bool HpnnSamples::get(size_t i, DOUBLE **in, DOUBLE **out) const {
    *in = *out = NULL;
    if (i >= names.size()) return false;
    if (!packed) {
        std::string p = dir + "/" + names[i];
        return _NN(read, sample)((CHAR *)p.c_str(), in, out);
    }
    *in = (DOUBLE *)malloc(sizeof(DOUBLE) * n_in);
    *out = (DOUBLE *)malloc(sizeof(DOUBLE) * n_out);
    memcpy(*in, X.data() + i * n_in, sizeof(DOUBLE) * n_in);
    memcpy(*out, T.data() + i * n_out, sizeof(DOUBLE) * n_out);
    return true;
}

size_t HpnnSamples::load(const std::vector<UINT> &order, UINT ni, UINT no, int threads, std::vector<DOUBLE> &Xo,
                         std::vector<DOUBLE> &To) const {
    Xo.clear();
    To.clear();
    if (!packed) return load_dir(dir, names, order, ni, no, threads, Xo, To, nullptr);
    if (ni != n_in || no != n_out) {
        NN_ERROR(stderr, "pack file holds %u -> %u samples, the network is %u -> %u\n", n_in, n_out, ni, no);
        return 0;
    }
    Xo.resize(order.size() * (size_t)ni);
    To.resize(order.size() * (size_t)no);
    for (size_t j = 0; j < order.size(); j++) {
        memcpy(Xo.data() + j * ni, X.data() + (size_t)order[j] * ni, sizeof(DOUBLE) * ni);
        memcpy(To.data() + j * no, T.data() + (size_t)order[j] * no, sizeof(DOUBLE) * no);
    }
    return order.size();
}

/* write n records from memory: the same pack file (names "s%08u"), for data generated in a
 * program (synthetic benchmark sets) rather than read from sample files */
static BOOL write_pack(const CHAR *filename, const std::vector<std::string> &names, const DOUBLE *X, const DOUBLE *T,
                       UINT n, UINT ni, UINT no) {
    std::string nm;
    for (const auto &s : names) {
        nm += s;
        nm.push_back('\0');
    }
    FILE *fp = fopen(filename, "wb");
    if (!fp) {
        NN_ERROR(stderr, "can't write pack file %s\n", filename);
        return FALSE;
    }
    const UINT hdr[4] = {n, ni, no, 0};
    const UINT64 nb = nm.size();
    const size_t nx = (size_t)n * ni, nt = (size_t)n * no;
    UINT64 h = hpnn_fnv1a(X, nx * 8, HPNN_FNV_SEED);
    h = hpnn_fnv1a(T, nt * 8, h);
    bool ok = fwrite(HPNN_PACK_MAGIC, 1, 8, fp) == 8 && fwrite(hdr, 4, 4, fp) == 4 && fwrite(&nb, 8, 1, fp) == 1 &&
              (nb == 0 || fwrite(nm.data(), 1, nb, fp) == nb) && fwrite(X, 8, nx, fp) == nx &&
              fwrite(T, 8, nt, fp) == nt && fwrite(&h, 8, 1, fp) == 1;
    ok = (fclose(fp) == 0) && ok;
    if (ok) NN_OUT(stdout, "packed %u samples (%u -> %u) into %s\n", n, ni, no, filename);
    return ok ? TRUE : FALSE;
}

extern "C" BOOL _NN(pack, arrays)(const CHAR *filename, const DOUBLE *X, const DOUBLE *T, UINT n, UINT n_in,
                                  UINT n_out) {
    if (!filename || !X || !T || n == 0 || n_in == 0 || n_out == 0) return FALSE;
    std::vector<std::string> names(n);
    char b[32];
    for (UINT i = 0; i < n; i++) {
        snprintf(b, sizeof b, "s%08u", i);
        names[i] = b;
    }
    return write_pack(filename, names, X, T, n, n_in, n_out);
}

extern "C" BOOL _NN(pack, samples)(const CHAR *dir, const CHAR *filename) {
    HpnnSamples s;
    if (!dir || !filename || !s.open(dir) || s.packed) {
        NN_ERROR(stderr, "can't open sample directory: %s\n", dir ? dir : "(null)");
        return FALSE;
    }
    std::vector<UINT> order(s.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = (UINT)i;
    std::vector<DOUBLE> X, T;
    std::vector<std::string> kept;
    UINT ni = 0, no = 0;
    if (load_dir(s.dir, s.names, order, ni, no, omp_get_max_threads(), X, T, &kept) == 0) return FALSE;
    return write_pack(filename, kept, X.data(), T.data(), (UINT)kept.size(), ni, no);
}
