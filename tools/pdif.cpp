/*
 * pdif -- RRUFF powder-XRD records (DIF + raw XY) -> libhpnn sample files.
 *
 * Parity with the reference tutorial tool (tutorials/ann/prepare_dif.c,
 * file_dif.c:37-478):
 *   usage: pdif RRUFF_DIR -i N_BINS -o N_OUT [-s SAMPLE_DIR]   (default ./samples)
 *   for every file F in RRUFF_DIR/dif/:
 *     - parse the DIF record: temperature from the "Sample ... T = v [K|C]" line
 *       (default 25 C; no K unit -> Celsius), "CELL PARAMETERS:" (6 numbers),
 *       "SPACE GROUP" (Hermann-Mauguin symbol -> international number, 0 if
 *       unknown), the ATOM block, "WAVELENGTH", the "2-THETA" peak list (at least
 *       one peak, else the record is skipped); records whose first line names
 *       R060187 or holds "5.000" are skipped (incomplete in the database)
 *     - skip records measured at lambda = 0.710730 (Mo radiation)
 *     - read RRUFF_DIR/raw/F: header lines until one starts with a digit, then
 *       "2theta, intensity" pairs (unparseable lines are skipped)
 *     - write SAMPLE_DIR/F:  "[input] N_BINS+1", T/273.15 followed by the raw
 *       intensity integrated over N_BINS equal 2theta bins of [5, 90) degrees and
 *       normalised by the largest bin ("%7.5f"), then "[output] N_OUT" and the +1/-1
 *       one-hot space group (position space-1; all -1 when unknown).
 * Differences from the reference: no read past the end of the raw arrays, files
 * are processed in sorted order (directory order is filesystem dependent), and a
 * summary line reports written / skipped counts.
 */
#include <dirent.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>
#include <cctype>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

constexpr double TH_MIN = 5.0, TH_MAX = 90.0;

/* international number -> accepted Hermann-Mauguin spellings (standard and the
 * alternative settings / axis choices that occur in RRUFF records) */
const std::pair<int, const char *> kSpaceGroups[] = {
    {1, "P1 C1 I1"}, {2, "P-1 A-1 B-1 C-1 F-1 I-1"}, {3, "P2"}, {4, "P2_1 B2_1 C2_1"},
    {5, "C2 A2 B2 F2 I2 I2_1"}, {6, "Pm"}, {7, "Pc Pa Pn Pb Bd Ca"}, {8, "Cm Am Im"},
    {9, "Cc Aa An Bb Cn Fd Ia Ic"}, {10, "P2/m"}, {11, "P2_1/m B2_1/m"},
    {12, "C2/m A2/m B2/m C2/a F2/m I2/m"}, {13, "P2/c C2/b P2/b P2/n P2/a"},
    {14, "P2_1/c B2_1/a B2_1/c B2_1/d P2_1/a P2_1/b P2_1/n"},
    {15, "C2/c A2/a A2/n B2_1/b B2/b B2/n C2/n F2/d I2/a I2/b I2/c I2/n I2_1/a I2_1/c"},
    {16, "P222"}, {17, "P222_1 P2_122 P22_12"}, {18, "P2_12_12 P2_122_1 P22_12_1"}, {19, "P2_12_12_1"},
    {20, "C222_1 A2_122 B22_12 C2_12_12_1"}, {21, "C222 A222 B222 C2_12_12"}, {22, "F222 F2_12_12_1"},
    {23, "I222"}, {24, "I2_12_12_1"}, {25, "Pmm2 Pm2m P2mm"},
    {26, "Pmc2_1 Pb2_1m Pcm2_1 Pm2_1b P2_1am P2_1ma"}, {27, "Pcc2 Pb2b P2aa"},
    {28, "Pma2 Pbm2 Pc2m Pm2a P2cm P2mb"}, {29, "Pca2_1 Pbc2_1 Pb2_1a Pc2_1b P2_1ab P2_1ca"},
    {30, "Pnc2 Pb2n Pcn2 Pn2b P2an P2na"}, {31, "Pmn2_1 Pm2_1n Pnm2_1 Pn2_1m P2_1mn P2_1nm"},
    {32, "Pba2 Pc2a P2cb"}, {33, "Pna2_1 Pbn2_1 Pc2_1n Pn2_1a P2_1cn P2_1nb"}, {34, "Pnn2 Pn2n P2nn"},
    {35, "Cmm2 A2mm Bm2m"}, {36, "Cmc2_1 A2_1am A2_1ma Bb2_1m Bm2_1b Ccm2_1 Cbn2_1"},
    {37, "Ccc2 A2aa Bb2b Cnn2"}, {38, "Amm2 Am2m Anc2_1 Bmm2 B2mm Cm2m C2mm"},
    {39, "Aem2 Abm2 Ab2m Acc2_1 Bma2 B2am Cm2a C2ma C2mb"},
    {40, "Ama2 Am2a Ann2_1 Bbm2 B2mb Cc2m C2cm"},
    {41, "Aea2 Aba2 Ab2a Acn2_1 Ac2a Bba2 B2ab Cc2a Cc2b C2ca C2cb"},
    {42, "Fmm2 Fm2m Fnn2 F2mm Fbc2_1 Fca2_1"}, {43, "Fdd2 Fd2d F2dd Fdd2_1"},
    {44, "Imm2 Im2m Inn2_1 I2mm"}, {45, "Iba2 Ib2a Icc2_1 Ic2a I2aa I2cb"},
    {46, "Ima2 Ibm2 Ib2m Im2a Inc2_1 I2am I2cm I2ma Pn2a"}, {47, "Pmmm"}, {48, "Pnnn"},
    {49, "Pccm Pbmb Pmaa"}, {50, "Pban Pcna Pncb"}, {51, "Pmma Pbmm Pcmm Pmam Pmcm Pmmb"},
    {52, "Pnna Pbnn Pcnn Pnan Pncn Pnnb"}, {53, "Pmna Pbmn Pcnm Pman Pncm Pnmb"},
    {54, "Pcca Pbaa Pbab Pbcb Pcaa Pccb"}, {55, "Pbam Pcma Pmcb"}, {56, "Pccn Pbnb Pnaa"},
    {57, "Pbcm Pbma Pcam Pcmb Pmab Pmca"}, {58, "Pnnm Pmnn Pnmn"}, {59, "Pmmn Pmnm Pnmm"},
    {60, "Pbcn Pbna Pcan Pcnb Pnab Pnca"}, {61, "Pbca Pcab"}, {62, "Pnma Pbnm Pcmn Pmcn Pmnb Pnam"},
    {63, "Cmcm Amam Amma Bbmm Bmmb Ccmm Cbnn"}, {64, "Cmce Abam Abma Acam Bbam Bbcm Bmab Cbnb Ccma Ccmb Cmca"},
    {65, "Cmmm Ammm Bmmm Cban"}, {66, "Cccm Amaa Bbmb Cnnn"}, {67, "Cmme Abmm Bmam Cbab Cmma"},
    {68, "Ccce Abaa Bbab Ccca Cnnb"}, {69, "Fmmm Fnnn"}, {70, "Fddd"}, {71, "Immm Innn"},
    {72, "Ibam Ibma Iccn Imaa Imcb"}, {73, "Ibca Icab"}, {74, "Imma Ibmm Imam Imcm Innb"},
    {75, "P4"}, {76, "P4_1"}, {77, "P4_2"}, {78, "P4_3"}, {79, "I4"}, {80, "I4_1"}, {81, "P-4"},
    {82, "I-4"}, {83, "P4/m"}, {84, "P4_2/m"}, {85, "P4/n"}, {86, "P4_2/n"}, {87, "I4/m"},
    {88, "I4_1/a"}, {89, "P422"}, {90, "P42_12"}, {91, "P4_122"}, {92, "P4_12_12 C4_122_1"},
    {93, "P4_222"}, {94, "P4_22_12"}, {95, "P4_322"}, {96, "P4_32_12"}, {97, "I422"}, {98, "I4_122"},
    {99, "P4mm"}, {100, "P4bm"}, {101, "P4_2cm"}, {102, "P4_2nm"}, {103, "P4cc"}, {104, "P4nc"},
    {105, "P4_2mc"}, {106, "P4_2bc"}, {107, "I4mm"}, {108, "I4cm"}, {109, "I4_1md"}, {110, "I4_1cd"},
    {111, "P-42m"}, {112, "P-42c"}, {113, "P-42_1m"}, {114, "P-42_1c"}, {115, "P-4m2"},
    {116, "P-4c2"}, {117, "P-4b2"}, {118, "P-4n2"}, {119, "I-4m2"}, {120, "I-4c2"}, {121, "I-42m"},
    {122, "I-42d"}, {123, "P4/mmm"}, {124, "P4/mcc"}, {125, "P4/nbm"}, {126, "P4/nnc"},
    {127, "P4/mbm"}, {128, "P4/mnc"}, {129, "P4/nmm"}, {130, "P4/ncc"}, {131, "P4_2/mmc"},
    {132, "P4_2/mcm"}, {133, "P4_2/nbc"}, {134, "P4_2/nnm"}, {135, "P4_2/mbc"}, {136, "P4_2/mnm"},
    {137, "P4_2/nmc"}, {138, "P4_2/ncm"}, {139, "I4/mmm"}, {140, "I4/mcm"}, {141, "I4_1/amd"},
    {142, "I4_1/acd"}, {143, "P3"}, {144, "P3_1"}, {145, "P3_2"}, {146, "R3 R3r"}, {147, "P-3"},
    {148, "R-3 R-3r"}, {149, "P312"}, {150, "P321"}, {151, "P3_112"}, {152, "P3_121"},
    {153, "P3_212"}, {154, "P3_221"}, {155, "R32 R32r"}, {156, "P3m1"}, {157, "P31m"},
    {158, "P3c1"}, {159, "P31c"}, {160, "R3m R3mr"}, {161, "R3c R3cr"}, {162, "P-31m"},
    {163, "P-31c"}, {164, "P-3m1"}, {165, "P-3c1"}, {166, "R-3m R-3mr"}, {167, "R-3c R-3cr"},
    {168, "P6"}, {169, "P6_1"}, {170, "P6_5"}, {171, "P6_2"}, {172, "P6_4"}, {173, "P6_3"},
    {174, "P-6"}, {175, "P6/m"}, {176, "P6_3/m"}, {177, "P622"}, {178, "P6_122"}, {179, "P6_522"},
    {180, "P6_222"}, {181, "P6_422"}, {182, "P6_322"}, {183, "P6mm"}, {184, "P6cc"}, {185, "P6_3cm"},
    {186, "P6_3mc"}, {187, "P-6m2"}, {188, "P-6c2"}, {189, "P-62m"}, {190, "P-62c"}, {191, "P6/mmm"},
    {192, "P6/mcc"}, {193, "P6_3/mcm"}, {194, "P6_3/mmc"}, {195, "P23"}, {196, "F23"}, {197, "I23"},
    {198, "P2_13"}, {199, "I2_13"}, {200, "Pm-3 Pm3"}, {201, "Pn-3 Pn3"}, {202, "Fm-3 Fm3"},
    {203, "Fd-3 Fd3"}, {204, "Im-3 Im3"}, {205, "Pa-3 Pa3 Pb3 Pb-3"}, {206, "Ia-3 Ia3"}, {207, "P432"},
    {208, "P4_232"}, {209, "F432"}, {210, "F4_132"}, {211, "I432"}, {212, "P4_332"}, {213, "P4_132"},
    {214, "I4_132"}, {215, "P-43m"}, {216, "F-43m"}, {217, "I-43m"}, {218, "P-43n"}, {219, "F-43c"},
    {220, "I-43d"}, {221, "Pm-3m Pm3m"}, {222, "Pn-3n Pn3n"}, {223, "Pm-3n Pm3n"}, {224, "Pn-3m Pn3m"},
    {225, "Fm-3m Fm3m"}, {226, "Fm-3c Fm3c"}, {227, "Fd-3m Fd3m"}, {228, "Fd-3c Fd3c"},
    {229, "Im-3m Im3m"}, {230, "Ia-3d Ia3d"}};

const std::unordered_map<std::string, int> &space_group_table() {
    static std::unordered_map<std::string, int> t = [] {
        std::unordered_map<std::string, int> m;
        for (const auto &e : kSpaceGroups) {
            std::istringstream in(e.second);
            std::string sym;
            while (in >> sym) m.emplace(sym, e.first);
        }
        return m;
    }();
    return t;
}

struct Record {
    double temp = 273.15 + 25.0; /* Kelvin */
    double cell[6] = {0, 0, 0, 0, 0, 0};
    int space = 0;
    int natoms = 0;
    double lambda = 1.541838;
    int n_peaks = 0;
    std::vector<double> raw_t, raw_i;
};

/* parse leading doubles separated by blanks / commas; returns how many were read */
int read_numbers(const char *p, double *out, int n) {
    int k = 0;
    while (k < n && *p) {
        while (*p && (isspace((unsigned char)*p) || *p == ',')) p++;
        if (!*p) break;
        char *end = nullptr;
        const double v = strtod(p, &end);
        if (end == p) break;
        out[k++] = v;
        p = end;
    }
    return k;
}

const char *skip_blank(const char *p) {
    while (*p && isspace((unsigned char)*p)) p++;
    return p;
}

bool read_lines(const std::string &path, std::vector<std::string> &lines) {
    FILE *f = fopen(path.c_str(), "r");
    if (!f) return false;
    char buf[4096];
    while (fgets(buf, sizeof buf, f)) lines.emplace_back(buf);
    fclose(f);
    return true;
}

/* 0: ok, 1: unreadable, 2: incomplete record */
int parse_dif(const std::string &path, Record &r) {
    std::vector<std::string> L;
    if (!read_lines(path, L) || L.empty()) return 1;
    if (L[0].find("R060187") != std::string::npos || L[0].find("5.000") != std::string::npos) return 2;
    for (size_t i = 1; i < L.size(); i++) {
        const std::string &ln = L[i];
        if (ln.find("Sample") != std::string::npos) {
            const size_t p = ln.find("T =");
            if (p != std::string::npos) {
                char *end = nullptr;
                const char *s = ln.c_str() + p + 3;
                const double v = strtod(s, &end);
                if (end != s) {
                    const char *u = skip_blank(end);
                    r.temp = (*u == 'K') ? v : v + 273.15;
                }
            }
        }
        size_t p = ln.find("CELL PARAMETERS:");
        if (p != std::string::npos && read_numbers(ln.c_str() + p + 16, r.cell, 6) != 6) return 2;
        p = ln.find("SPACE GROUP");
        if (p != std::string::npos) {
            const char *s = ln.c_str() + p + 11;
            while (*s && *s != ':') s++; /* "SPACE GROUP:" and the odd "SPACE GROUP #:" */
            if (*s == ':') s++;
            s = skip_blank(s);
            std::string sym;
            while (*s && !isspace((unsigned char)*s)) sym.push_back(*s++);
            const auto &t = space_group_table();
            const auto it = t.find(sym);
            r.space = it == t.end() ? 0 : it->second;
        }
        if (ln.find("ATOM") != std::string::npos) {
            /* atom lines: symbol then x y z occupancy B, until a line starting with a digit or blank */
            for (i++; i < L.size(); i++) {
                const char *s = skip_blank(L[i].c_str());
                if (!*s || isdigit((unsigned char)*s) || !isgraph((unsigned char)*s)) break;
                while (*s && !isspace((unsigned char)*s)) s++;
                double v[5];
                if (read_numbers(s, v, 5) != 5) return 2;
                r.natoms++;
            }
            if (i < L.size()) i--; /* re-examine the line that ended the block */
            continue;
        }
        p = ln.find("WAVELENGTH");
        if (p != std::string::npos) {
            const char *s = ln.c_str() + p;
            while (*s && !isdigit((unsigned char)*s)) s++;
            if (*s) r.lambda = strtod(s, nullptr);
        }
        if (ln.find("2-THETA") != std::string::npos) {
            for (i++; i < L.size(); i++) {
                const char *s = L[i].c_str();
                while (*s && *s != '\n' && !isdigit((unsigned char)*s)) s++;
                if (!isdigit((unsigned char)*s)) break;
                double v[2];
                if (read_numbers(s, v, 2) != 2) return 2;
                r.n_peaks++;
            }
            if (i < L.size()) i--;
        }
    }
    return r.n_peaks > 0 ? 0 : 2;
}

bool parse_raw(const std::string &path, Record &r) {
    std::vector<std::string> L;
    if (!read_lines(path, L)) return false;
    size_t i = 0;
    while (i < L.size() && !isdigit((unsigned char)L[i][0])) i++;
    if (i == L.size()) return false;
    for (; i < L.size(); i++) {
        double v[2];
        if (read_numbers(L[i].c_str(), v, 2) != 2) continue; /* permissive, like the reference */
        r.raw_t.push_back(v[0]);
        r.raw_i.push_back(v[1]);
    }
    return true;
}

bool write_sample(const std::string &path, const Record &r, int n_bins, int n_out) {
    std::vector<double> bins(n_bins, 0.0);
    const double width = (TH_MAX - TH_MIN) / n_bins;
    size_t j = 0;
    const size_t n = r.raw_t.size();
    while (j < n && r.raw_t[j] < TH_MIN) j++;
    double upper = TH_MIN + width, vmax = 0.0;
    for (int b = 0; b < n_bins; b++, upper += width) {
        double acc = 0.0;
        while (j < n && r.raw_t[j] < upper) acc += r.raw_i[j++];
        bins[b] = acc;
        vmax = std::max(vmax, acc);
    }
    if (vmax == 0.0) return false;
    FILE *f = fopen(path.c_str(), "w");
    if (!f) return false;
    fprintf(f, "[input] %d\n%7.5f", n_bins + 1, r.temp / 273.15);
    for (int b = 0; b < n_bins; b++) fprintf(f, " %7.5f", bins[b] / vmax);
    fprintf(f, "\n[output] %d\n", n_out);
    for (int o = 0; o < n_out; o++) fprintf(f, "%s%s", o ? " " : "", (o == r.space - 1) ? "1.0" : "-1.0");
    fprintf(f, "\n");
    fclose(f);
    return true;
}

void usage(FILE *o) {
    fprintf(o,
            "usage: pdif RRUFF_DIR -i N_BINS -o N_OUT [-s SAMPLE_DIR]\n"
            "  RRUFF_DIR   directory holding dif/ and raw/ (same file names)\n"
            "  -i N_BINS   2theta bins in [5,90) deg; the network gets N_BINS+1 inputs\n"
            "              (the first one is the relative temperature T/273.15)\n"
            "  -o N_OUT    outputs (230 space groups)\n"
            "  -s DIR      where the sample files go (default ./samples)\n");
}

bool int_arg(int argc, char **argv, int &i, int j, int &out) {
    const char *s = argv[i] + j + 1;
    if (!*s) {
        if (++i >= argc) return false;
        s = argv[i];
    }
    char *end = nullptr;
    const long v = strtol(s, &end, 10);
    if (end == s || *end || v <= 0) return false;
    out = (int)v;
    return true;
}

}  // namespace

int main(int argc, char **argv) {
    std::string rruff, samples = "./samples";
    int n_bins = 0, n_out = 0;
    for (int i = 1; i < argc; i++) {
        const char *a = argv[i];
        if (a[0] == '-' && a[1]) {
            bool ok = true;
            switch (a[1]) {
            case 'h':
                usage(stdout);
                return 0;
            case 'i': ok = int_arg(argc, argv, i, 1, n_bins); break;
            case 'o': ok = int_arg(argc, argv, i, 1, n_out); break;
            case 's':
                if (a[2]) samples = a + 2;
                else if (i + 1 < argc) samples = argv[++i];
                else ok = false;
                break;
            default: ok = false;
            }
            if (!ok) {
                fprintf(stderr, "syntax error near '%s'\n", a);
                usage(stderr);
                return 1;
            }
        } else if (rruff.empty()) {
            rruff = a;
        } else {
            fprintf(stderr, "syntax error: too many parameters\n");
            usage(stderr);
            return 1;
        }
    }
    if (rruff.empty() || n_bins <= 0 || n_out <= 0) {
        usage(stderr);
        return 1;
    }
    fprintf(stdout, ">> received: %s -i %d -o %d -s %s\n", rruff.c_str(), n_bins + 1, n_out, samples.c_str());
    struct stat st;
    if (stat(samples.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) {
        fprintf(stderr, "ERROR: can't open directory: %s\n", samples.c_str());
        return 1;
    }
    const std::string difdir = rruff + "/dif/";
    DIR *d = opendir(difdir.c_str());
    if (!d) {
        fprintf(stderr, "ERROR: can't open directory: %s\n", difdir.c_str());
        return 1;
    }
    std::vector<std::string> files;
    while (struct dirent *e = readdir(d))
        if (e->d_name[0] != '.') files.emplace_back(e->d_name);
    closedir(d);
    std::sort(files.begin(), files.end());
    int written = 0, skipped = 0;
    for (const auto &f : files) {
        fprintf(stdout, "Processing file: %s\n", f.c_str());
        Record r;
        const int rc = parse_dif(difdir + f, r);
        if (rc) {
            fprintf(stderr, "ERROR: reading %s file! SKIP\n", f.c_str());
            skipped++;
            continue;
        }
        if (r.lambda == 0.710730) {
            fprintf(stderr, "ERROR: file %s has wavelength of 0.710730! SKIP\n", f.c_str());
            skipped++;
            continue;
        }
        if (!parse_raw(rruff + "/raw/" + f, r)) {
            fprintf(stderr, "ERROR: reading %s/raw/%s file! SKIP\n", rruff.c_str(), f.c_str());
            skipped++;
            continue;
        }
        if (!write_sample(samples + "/" + f, r, n_bins, n_out)) {
            fprintf(stderr, "ERROR: writing %s sample file!\n", f.c_str());
            skipped++;
            continue;
        }
        written++;
    }
    fprintf(stdout, ">> %d samples written, %d records skipped\n", written, skipped);
    return 0;
}
