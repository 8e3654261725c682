/*
 * File-based launcher bootstrap (include/libhpnn/bootstrap.h).
 *
 * The reference's MPI tier got rank, size and collectives from MPI_Init
 * (libhpnn.c:182-200).  Without libmpi, the native multi-process path needs only a few
 * host-side exchanges per run, so a directory on the node's filesystem does: rank r
 * writes <seq>.<r> (temporary name + rename, so a reader never sees a torn file) and
 * polls for the others.
 */
#include <libhpnn.h>
#include <libhpnn/bootstrap.h>
#include <dirent.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <string>
#include <thread>
#include <vector>

namespace {

int g_seq = 0;
const time_t g_start = time(nullptr);

int env_int(const char *n, int d) {
    const char *e = getenv(n);
    return e ? atoi(e) : d;
}

std::string boot_dir() {
    const char *d = getenv("HPNN_BOOT_DIR");
    if (d && d[0]) return d;
    const char *t = getenv("TMPDIR");
    const char *a = getenv("MASTER_ADDR"), *p = getenv("MASTER_PORT"), *r = getenv("TORCHELASTIC_RUN_ID");
    std::string s = std::string("hpnn_boot_") + (a ? a : "local") + "_" + (p ? p : "0") + "_" + (r ? r : "run");
    for (char &c : s)
        if (c == ':' || c == '/') c = '_';
    return std::string(t && t[0] ? t : "/tmp") + "/" + s;
}

std::string file_of(const std::string &dir, int seq, int rank) {
    return dir + "/" + std::to_string(seq) + "." + std::to_string(rank);
}

bool read_file(const std::string &path, void *dst, size_t n) {
    FILE *fp = fopen(path.c_str(), "rb");
    if (!fp) return false;
    const bool ok = fread(dst, 1, n, fp) == n;
    fclose(fp);
    return ok;
}

}  // namespace

extern "C" int hpnn_boot_rank(void) { return env_int("RANK", 0); }
extern "C" int hpnn_boot_world(void) { return env_int("WORLD_SIZE", 1); }

extern "C" int hpnn_boot_allgather(const void *mine, size_t n, void *all) {
    const int rank = hpnn_boot_rank(), world = hpnn_boot_world();
    const int seq = g_seq++;
    if (world <= 1) {
        memcpy(all, mine, n);
        return 0;
    }
    const std::string dir = boot_dir();
    mkdir(dir.c_str(), 0700); /* EEXIST from the other ranks is fine */
    const std::string mine_path = file_of(dir, seq, rank);
    {
        const std::string tmp = mine_path + ".tmp";
        FILE *fp = fopen(tmp.c_str(), "wb");
        if (!fp) {
            NN_ERROR(stderr, "bootstrap: can't write %s (%s)\n", tmp.c_str(), strerror(errno));
            return -2;
        }
        const bool ok = fwrite(mine, 1, n, fp) == n;
        if (fclose(fp) != 0 || !ok || rename(tmp.c_str(), mine_path.c_str()) != 0) return -2;
    }
    const double timeout = env_int("HPNN_BOOT_TIMEOUT_S", 120);
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < world; r++) {
        const std::string path = file_of(dir, seq, r);
        struct stat st;
        for (;;) {
            if (stat(path.c_str(), &st) == 0 && (size_t)st.st_size == n && st.st_mtime >= g_start - 120) break;
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout) {
                NN_ERROR(stderr, "bootstrap: rank %d waited %.0f s for rank %d (%s)\n", rank, timeout, r,
                         path.c_str());
                return -3;
            }
            /* fine polling first: in training loops the ranks arrive within microseconds */
            const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            std::this_thread::sleep_for(std::chrono::microseconds(waited < 0.05 ? 20 : 2000));
        }
        if (!read_file(path, (char *)all + (size_t)r * n, n)) return -2;
    }
    return 0;
}

extern "C" void hpnn_boot_finish(void) {
    const int world = hpnn_boot_world();
    if (world <= 1) return;
    std::vector<char> all((size_t)world);
    char z = 0;
    if (hpnn_boot_allgather(&z, 1, all.data()) != 0) return;
    const int a = g_seq - 1; /* after barrier b every rank has read every file up to a */
    if (hpnn_boot_allgather(&z, 1, all.data()) != 0) return;
    if (hpnn_boot_rank() != 0) return;
    const std::string dir = boot_dir();
    for (int s = 0; s <= a; s++)
        for (int r = 0; r < world; r++) unlink(file_of(dir, s, r).c_str());
}
