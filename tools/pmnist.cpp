/*
 * pmnist -- convert MNIST IDX files into libhpnn sample files.
 *
 * Parity: reference tutorials/mnist/prepare_mnist.c (reads ./train_images,
 * ./train_labels, ./test_images, ./test_labels; writes one file per image,
 * s%05d.txt, "[input] 784" + pixels, "[output] 10 #label" + one-hot).
 * Fixed reference quirks: the first test label is read once
 * (labels were shifted by one), test files are numbered from 1.
 * Options:
 *   -n        normalise pixels to [0,1] (reference writes raw 0..255)
 *   -s        SNN targets 1/0 (reference writes +1/-1)
 *   -g NTR NTE  no IDX input: write NTR/NTE synthetic MNIST-shaped samples
 *             (class-dependent blobs + noise; for machines without the data)
 *   -p DIR    directory holding the IDX files (default .)
 */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include <string>
#include <vector>

static uint32_t be32(const unsigned char *b) { return ((uint32_t)b[0] << 24) | (b[1] << 16) | (b[2] << 8) | b[3]; }

static bool read_idx(const std::string &path, std::vector<unsigned char> &data, uint32_t &count, uint32_t &rows,
                     uint32_t &cols, bool images) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) {
        fprintf(stderr, "FAILED to open %s for READ!\n", path.c_str());
        return false;
    }
    unsigned char hdr[16];
    size_t hl = images ? 16 : 8;
    if (fread(hdr, 1, hl, f) != hl) {
        fclose(f);
        return false;
    }
    count = be32(hdr + 4);
    rows = images ? be32(hdr + 8) : 1;
    cols = images ? be32(hdr + 12) : 1;
    data.resize((size_t)count * rows * cols);
    size_t got = fread(data.data(), 1, data.size(), f);
    fclose(f);
    if (got != data.size()) {
        fprintf(stderr, "%s: truncated (%zu of %zu bytes)\n", path.c_str(), got, data.size());
        return false;
    }
    return true;
}

static void write_sample(const std::string &path, const float *px, int npx, int label, bool snn) {
    FILE *f = fopen(path.c_str(), "w");
    if (!f) {
        fprintf(stderr, "FAILED to open sample %s for WRITE!\n", path.c_str());
        exit(1);
    }
    fprintf(f, "[input] %d\n", npx);
    fprintf(f, "%7.5f", px[0]);
    for (int i = 1; i < npx; i++) fprintf(f, " %7.5f", px[i]);
    fprintf(f, "\n[output] %d  #%d\n", 10, label);
    const char *hi = "1.0", *lo = snn ? "0.0" : "-1.0";
    for (int i = 0; i < 10; i++) fprintf(f, i ? " %s" : "%s", i == label ? hi : lo);
    fprintf(f, "\n");
    fclose(f);
}

static int convert(const std::string &dir, const char *img, const char *lab, const std::string &out, bool norm,
                   bool snn) {
    std::vector<unsigned char> im, lb;
    uint32_t n, r, c, nl, r1, c1;
    if (!read_idx(dir + "/" + img, im, n, r, c, true)) return -1;
    if (!read_idx(dir + "/" + lab, lb, nl, r1, c1, false)) return -1;
    if (n != nl) {
        fprintf(stderr, "ERROR: different set size! %u vs %u\n", n, nl);
        return -1;
    }
    const int npx = (int)(r * c);
    std::vector<float> px(npx);
    for (uint32_t i = 0; i < n; i++) {
        if (lb[i] > 9) {
            fprintf(stderr, "ERROR: label out of boundaries!\n");
            continue;
        }
        for (int p = 0; p < npx; p++) px[p] = norm ? im[(size_t)i * npx + p] / 255.0f : (float)im[(size_t)i * npx + p];
        char name[32];
        snprintf(name, sizeof(name), "/s%05u.txt", i + 1);
        write_sample(out + name, px.data(), npx, lb[i], snn);
    }
    printf("# wrote %u samples to %s\n", n, out.c_str());
    return 0;
}

static void synth(const std::string &out, int n, unsigned seed, bool norm, bool snn) {
    srandom(seed);
    std::vector<float> px(784);
    for (int i = 0; i < n; i++) {
        int label = (int)(random() % 10);
        for (int p = 0; p < 784; p++) {
            int y = p / 28, x = p % 28;
            /* one bright 7x7 blob per class on a 4x3 grid, plus noise */
            int cy = 4 + (label / 3) * 7, cx = 4 + (label % 3) * 9;
            float v = (abs(y - cy) < 4 && abs(x - cx) < 4) ? 200.f : 0.f;
            v += (float)(random() % 56);
            px[p] = norm ? v / 255.f : v;
        }
        char name[32];
        snprintf(name, sizeof(name), "/s%05d.txt", i + 1);
        write_sample(out + name, px.data(), 784, label, snn);
    }
    printf("# wrote %d synthetic samples to %s\n", n, out.c_str());
}

int main(int argc, char *argv[]) {
    bool norm = false, snn = false;
    int gen_tr = -1, gen_te = -1;
    std::string dir = ".";
    std::vector<std::string> pos;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-n")) norm = true;
        else if (!strcmp(argv[i], "-s")) snn = true;
        else if (!strcmp(argv[i], "-g") && i + 2 < argc) {
            gen_tr = atoi(argv[++i]);
            gen_te = atoi(argv[++i]);
        } else if (!strcmp(argv[i], "-p") && i + 1 < argc) dir = argv[++i];
        else if (!strcmp(argv[i], "-h")) pos.clear(), argc = 0;
        else pos.push_back(argv[i]);
    }
    if (pos.size() != 2) {
        printf("usage: pmnist [-n] [-s] [-p idx_dir] [-g n_train n_test] samples_dir tests_dir\n");
        printf("IDX files: train_images train_labels test_images test_labels\n");
        return pos.empty() ? 0 : -1;
    }
    if (gen_tr >= 0) {
        synth(pos[0], gen_tr, 10958, norm, snn);
        synth(pos[1], gen_te, 10959, norm, snn);
        return 0;
    }
    if (convert(dir, "train_images", "train_labels", pos[0], norm, snn)) return -1;
    if (convert(dir, "test_images", "test_labels", pos[1], norm, snn)) return -1;
    return 0;
}
