/*
 * Python binding of the libhpnn HIP kernel launchers (pybind11).
 *
 * Deliberately torch-free: tensors cross the boundary as raw device
 * addresses (tensor.data_ptr()) and the HIP stream as an integer handle
 * (torch.cuda.current_stream().cuda_stream), so the module is a thin,
 * ABI-stable shim over libhpnn.so and every launch is captured by
 * torch.cuda.graph like any other kernel on that stream.
 */
#include <pybind11/pybind11.h>
#include <hip/hip_runtime_api.h>
#include <libhpnn.h>
#include <stdexcept>
#include <string>
#include <vector>
#include <tuple>
#include <pybind11/stl.h>

#include "../gpu/kernels.h"
#include "../gpu/bplan.h"
#include "../dist/dp_exchange.h"
#include <libhpnn/comm.h>
#include <libhpnn/xar.h>
#include <libhpnn/devmem.h>

namespace py = pybind11;
using uptr = uintptr_t;

static inline void *P(uptr p) { return reinterpret_cast<void *>(p); }
static inline hipStream_t S(uptr s) { return reinterpret_cast<hipStream_t>(s); }
static void check(int rc, const char *what) {
    if (rc != 0) throw std::runtime_error(std::string(what) + " failed (rc=" + std::to_string(rc) + ")");
}

namespace {
using hpnn::BPlan;
using hpnn::XIn;

XIn xin(uptr x, uptr xg, int u8, float scale) {
    XIn v;
    v.x = P(x);
    v.xg = P(xg);
    v.u8 = u8;
    v.scale = scale;
    return v;
}

/* the batched training plan (csrc/gpu/bplan.h): configuration + buffer table on the host,
 * launches on the given stream; memory is bound from tensors the caller allocated */
void bind_plan(py::module_ &m) {
    py::class_<BPlan>(m, "BPlan")
        .def(py::init([](std::vector<int> sizes, int type, int batch, bool momentum, int fused,
                         std::vector<int> splits, int mid_grid, bool device) {
                 auto *p = new BPlan();
                 std::string err;
                 if (sizes.size() < 2) throw std::runtime_error("BPlan: at least two layer sizes");
                 std::vector<int> sp(sizes.size(), 0);
                 for (size_t i = 0; i < splits.size() && i < sp.size(); i++) sp[i] = splits[i];
                 const int rc = p->configure(sizes.data(), (int)sizes.size() - 1, type, batch, momentum, fused,
                                             sp.data(), mid_grid, device, &err);
                 if (rc) {
                     delete p;
                     throw std::invalid_argument("BPlan: " + err + " (rc=" + std::to_string(rc) + ")");
                 }
                 return p;
             }),
             py::arg("sizes"), py::arg("type"), py::arg("batch"), py::arg("momentum"), py::arg("fused") = -1,
             py::arg("splits") = std::vector<int>(), py::arg("mid_grid") = 512, py::arg("device") = true)
        .def("config",
             [](const BPlan &p) {
                 py::dict d;
                 d["L"] = p.L;
                 d["Bp"] = p.Bp;
                 d["mode"] = p.mode ? std::string(1, p.mode) : std::string();
                 d["Kp"] = std::vector<int>(p.Kp, p.Kp + p.L);
                 d["Np"] = std::vector<int>(p.Np, p.Np + p.L);
                 d["S"] = std::vector<int>(p.S, p.S + p.L);
                 d["mid_grid"] = p.mid_grid;
                 d["mid_groups"] = p.mid_groups;
                 d["wide_ksplit"] = p.wide_ksplit;
                 d["slab_floats"] = p.slab_f;
                 d["input_layout"] = p.input_layout();
                 d["buckets"] = p.buckets();
                 return d;
             })
        .def("buffers",
             [](const BPlan &p) {
                 py::list out;
                 for (const auto &b : p.specs)
                     out.append(py::make_tuple(b.name, b.layer, b.dtype,
                                               std::vector<long>(b.shape, b.shape + b.ndim), b.zero));
                 return out;
             })
        .def("bind",
             [](BPlan &p, std::vector<uptr> ptrs) {
                 if (ptrs.size() != p.specs.size()) throw std::runtime_error("BPlan.bind: one pointer per buffer");
                 std::vector<void *> v;
                 for (uptr a : ptrs) v.push_back(P(a));
                 p.bind(v.data());
             })
        .def_static("pick_splits", &BPlan::pick_splits)
        .def("cast_weights", [](BPlan &p, uptr s) { check(p.cast_weights(S(s)), "BPlan.cast_weights"); })
        .def("zero_stats", [](BPlan &p, uptr s) { check(p.zero_stats(S(s)), "BPlan.zero_stats"); })
        .def("forward", [](BPlan &p, uptr X, uptr s) { check(p.forward(P(X), S(s)), "BPlan.forward"); })
        .def("output",
             [](BPlan &p, uptr labels, uptr T, int ldt, int n_valid, uptr O, int ldo, bool stats, uptr s) {
                 check(p.output((const int *)P(labels), (const float *)P(T), ldt, n_valid, (float *)P(O), ldo, stats,
                                S(s)),
                       "BPlan.output");
             })
        .def("backward_layer", [](BPlan &p, int l, uptr s) { check(p.backward_layer(l, S(s)), "BPlan.backward_layer"); })
        .def("grad_layer",
             [](BPlan &p, int l, uptr x, uptr xg, int u8, float sc, bool reduce, uptr s) {
                 check(p.grad_layer(l, xin(x, xg, u8, sc), reduce, S(s)), "BPlan.grad_layer");
             })
        .def("update_layer",
             [](BPlan &p, int l, float lr, float alpha, float scale, bool from_g, uptr s) {
                 check(p.update_layer(l, lr, alpha, scale, from_g, S(s)), "BPlan.update_layer");
             })
        .def("front",
             [](BPlan &p, uptr x, uptr xg, int u8, float sc, uptr labels, uptr T, int ldt, int n_valid, uptr s) {
                 check(p.front(xin(x, xg, u8, sc), (const int *)P(labels), (const float *)P(T), ldt, n_valid, S(s)),
                       "BPlan.front");
             })
        .def("step",
             [](BPlan &p, uptr x, uptr xg, int u8, float sc, uptr labels, uptr T, int ldt, int n_valid, float lr,
                float alpha, uptr s) {
                 check(p.step(xin(x, xg, u8, sc), (const int *)P(labels), (const float *)P(T), ldt, n_valid, lr, alpha,
                              S(s)),
                       "BPlan.step");
             })
        .def("grads",
             [](BPlan &p, uptr x, uptr xg, int u8, float sc, uptr labels, uptr T, int ldt, int n_valid,
                py::object ready, uptr s) {
                 hpnn::ReadyFn fn = [&](int lo, int hi) {
                     if (ready.is_none()) return true;
                     py::object r = ready(lo, hi);
                     return r.is_none() || r.cast<bool>();
                 };
                 check(p.grads(xin(x, xg, u8, sc), (const int *)P(labels), (const float *)P(T), ldt, n_valid, fn,
                               S(s)),
                       "BPlan.grads");
             })
        .def("grads_slabs",
             [](BPlan &p, uptr x, uptr xg, int u8, float sc, uptr labels, uptr T, int ldt, int n_valid, uptr s,
                uptr dst, uptr sel, long alt) {
                 hpnn::SlabSegs g;
                 check(p.grads_slabs(xin(x, xg, u8, sc), (const int *)P(labels), (const float *)P(T), ldt, n_valid,
                                     &g, S(s), (float *)P(dst), (const unsigned int *)P(sel), alt),
                       "BPlan.grads_slabs");
                 py::list out; /* (address, slab stride, slabs, floats) per segment */
                 for (int i = 0; i < g.count; i++)
                     out.append(py::make_tuple((uptr)g.base[i], g.stride[i], g.cnt[i], g.n[i]));
                 return out;
             })
        .def("xchg_step",
             [](BPlan &p, uptr x, uptr xg, int u8, float sc, uptr labels, uptr T, int ldt, int n_valid, float lr,
                float alpha, float scale, uptr xar, uptr s) {
                 hpnn_xar_view v;
                 check(hpnn_xar_view_get((hpnn_xar *)xar, &v), "xar_view_get");
                 const int r = p.xchg_step(xin(x, xg, u8, sc), (const int *)P(labels), (const float *)P(T), ldt,
                                           n_valid, lr, alpha, scale, v, S(s));
                 if (r != -1) check(r, "BPlan.xchg_step");
                 return r == 0;
             })
        .def("xchg_self_test",
             [](BPlan &p, uptr xar, uptr s) {
                 hpnn_xar_view v;
                 check(hpnn_xar_view_get((hpnn_xar *)xar, &v), "xar_view_get");
                 return p.xchg_self_test(v, S(s));
             })
        .def("update_flat",
             [](BPlan &p, uptr G, float lr, float alpha, float scale, uptr s) {
                 check(p.update_flat((const float *)P(G), lr, alpha, scale, S(s)), "BPlan.update_flat");
             })
        .def("health", [](BPlan &p, uptr s) { return p.health(S(s)); })
        .def("weights_digest",
             [](BPlan &p, int which, uptr s) {
                 unsigned long long d = 0;
                 check(p.weights_digest(which, &d, S(s)), "weights_digest");
                 return d;
             })
        .def_readwrite("g0_fused", &BPlan::g0_fused)
        .def_readwrite("g0_perm", &BPlan::g0_perm)
        .def_readwrite("g0_xcd", &BPlan::g0_xcd)
        .def_readwrite("tn_update", &BPlan::tn_update)
        .def_readwrite("tn8_side", &BPlan::tn8_side)
        .def_readwrite("side_launches", &BPlan::side_launches)
        .def_property_readonly("nn_bwd", [](const BPlan &p) { return std::vector<bool>(p.nn_bwd, p.nn_bwd + 16); })
        .def("tn_update_ok", &BPlan::tn_update_ok)
        .def("predict", [](BPlan &p, uptr X, int n_valid, uptr O, int ldo, uptr s) {
            check(p.predict(P(X), n_valid, (float *)P(O), ldo, S(s)), "BPlan.predict");
        });
}
/* native data-parallel step (csrc/dist/dp_exchange.h): keeps its plan alive */
void bind_dpx(py::module_ &m) {
    py::class_<hpnn::DpExchange>(m, "DpExchange")
        .def(py::init([](BPlan &plan, uptr comm, int mode) {
                 auto *d = new hpnn::DpExchange();
                 const int rc = d->init(&plan, (hpnn_comm *)comm, mode);
                 if (rc) {
                     delete d;
                     throw std::runtime_error("DpExchange init failed (rc=" + std::to_string(rc) + ")");
                 }
                 return d;
             }),
             py::keep_alive<1, 2>())
        .def("step",
             [](hpnn::DpExchange &d, uptr x, uptr xg, int u8, float sc, uptr labels, uptr T, int ldt, int n_valid,
                int n_total, float lr, float alpha, uptr s) {
                 check(d.step(xin(x, xg, u8, sc), (const int *)P(labels), (const float *)P(T), ldt, n_valid, n_total,
                              lr, alpha, S(s)),
                       "DpExchange.step");
             })
        .def("gather_masters", [](hpnn::DpExchange &d, uptr s) { check(d.gather_masters(S(s)), "gather_masters"); })
        .def("sharded", &hpnn::DpExchange::sharded);
}
}  // namespace

PYBIND11_MODULE(_native, m) {
    bind_plan(m);
    bind_dpx(m);
    m.doc() = "libhpnn gfx950 kernels (MFMA GEMMs, fused output/optimizer kernels)";
    m.attr("EPI_NONE") = (int)HPNN_EPI_NONE;
    m.attr("EPI_ACT") = (int)HPNN_EPI_ACT;
    m.attr("EPI_DACT") = (int)HPNN_EPI_DACT;

    m.def("version", []() { return std::string(nn_return_version()); });

    m.def(
        "gemm_nt_bf16",
        [](uptr A, int lda, uptr B, int ldb, uptr C, int ldc, uptr aux, int ldaux, int M, int N, int K, int epi,
           int c_f32, uptr stream) {
            check(hpnn_gemm_nt_bf16(P(A), lda, P(B), ldb, P(C), ldc, P(aux), ldaux, M, N, K, epi, c_f32, S(stream)),
                  "gemm_nt_bf16");
        },
        "C = epi(A . B^T), bf16 MFMA");
    m.def(
        "gemm_tn_bf16",
        [](uptr D, int ldd, uptr H, int ldh, uptr slab, int ldg, int N, int M, int Bt, int splits, uptr stream) {
            check(hpnn_gemm_tn_bf16(P(D), ldd, P(H), ldh, (float *)P(slab), ldg, N, M, Bt, splits, S(stream)),
                  "gemm_tn_bf16");
        },
        "slab[s] = D^T . H over batch slice s, bf16 MFMA");
    m.def(
        "output_delta",
        [](uptr Z, int ldz, uptr T, int ldt, uptr labels, float t_hi, float t_lo, uptr D, int ldd, uptr O, int ldo,
           uptr loss, uptr correct, int B, int n_valid, int n_out, int type, uptr stream) {
            check(hpnn_output_delta((const float *)P(Z), ldz, (const float *)P(T), ldt, (const int *)P(labels), t_hi,
                                    t_lo, P(D), ldd, (float *)P(O), ldo, (float *)P(loss), (unsigned int *)P(correct),
                                    B, n_valid, n_out, type, S(stream)),
                  "output_delta");
        });
    m.def("gemm_nt_set_8ph", [](int on) { hpnn_gemm_nt_set_8ph(on); });
    m.def("gemm_tn8_update", [](uptr D, int ldd, uptr H, int ldh, int N, int M, int Bt, uptr W32, uptr V32, uptr Wbf,
                                uptr Wt, float lr, float alpha, float scale, int momentum, uptr stream) {
        const int rc = hpnn_gemm_tn8_update(P(D), ldd, P(H), ldh, N, M, Bt, (float *)P(W32), (float *)P(V32), P(Wbf),
                                            P(Wt), lr, alpha, scale, momentum, S(stream));
        if (rc != -1) check(rc, "gemm_tn8_update");
        return rc == 0;
    });
    m.def("gemm_nt8_splitk_bf16", [](uptr A, int lda, uptr B, int ldb, uptr C, int ldc, uptr aux, int ldaux, int M,
                                     int N, int K, int epi, int c_f32, int splits, uptr stream) {
        check(hpnn_gemm_nt8_splitk_bf16(P(A), lda, P(B), ldb, P(C), ldc, P(aux), ldaux, M, N, K, epi, c_f32, splits,
                                        S(stream)),
              "gemm_nt8_splitk_bf16");
    });
    m.def("gemm_tn_set_8ph", [](int on) { hpnn_gemm_tn_set_8ph(on); });
    m.def("gemm_nt_set_pp", [](int on) { hpnn_gemm_nt_set_pp(on); });
    m.def(
        "gemm_nt8_bf16",
        [](uptr A, int lda, uptr B, int ldb, uptr C, int ldc, uptr aux, int ldaux, int M, int N, int K, int epi,
           int c_f32, uptr stream) {
            check(hpnn_gemm_nt8_bf16(P(A), lda, P(B), ldb, P(C), ldc, P(aux), ldaux, M, N, K, epi, c_f32, S(stream)),
                  "gemm_nt8_bf16");
        },
        "C = epi(A . B^T), bf16 MFMA");
    m.def(
        "gemm_nn_bf16",
        [](uptr A, int lda, uptr W, int ldw, uptr C, int ldc, uptr aux, int ldaux, int M, int N, int K, int epi,
           int c_f32, uptr stream) {
            check(hpnn_gemm_nn_bf16(P(A), lda, P(W), ldw, P(C), ldc, P(aux), ldaux, M, N, K, epi, c_f32, S(stream)),
                  "gemm_nn_bf16");
        },
        "C = epi(A . W), W row-major [K][N], bf16 MFMA");
    m.def("transpose_bf16", [](uptr Wb, uptr Wt, int N, int K, uptr stream) {
        check(hpnn_transpose_bf16(P(Wb), P(Wt), N, K, S(stream)), "transpose_bf16");
    });
    m.def("reduce_slabs", [](uptr slab, int Sn, long stride, long n, uptr out, uptr stream) {
        check(hpnn_reduce_slabs((const float *)P(slab), Sn, stride, n, (float *)P(out), S(stream)), "reduce_slabs");
    });
    m.def("sgd_update", [](uptr W32, uptr V32, uptr G, int Sn, long gstride, uptr Wbf, uptr Wt, int N, int K, float lr,
                           float alpha, float scale, int momentum, uptr stream) {
        check(hpnn_sgd_update((float *)P(W32), (float *)P(V32), (const float *)P(G), Sn, gstride, P(Wbf), P(Wt), N, K,
                              lr, alpha, scale, momentum, S(stream)),
              "sgd_update");
    });
    m.def("cast_weights", [](uptr W32, uptr Wbf, uptr Wt, int N, int K, uptr stream) {
        check(hpnn_cast_weights((const float *)P(W32), P(Wbf), P(Wt), N, K, S(stream)), "cast_weights");
    });
    m.def("block_permute_bf16", [](uptr src, uptr dst, int Pn, long rows, int n, uptr stream) {
        check(hpnn_block_permute_bf16(P(src), P(dst), Pn, rows, n, S(stream)), "block_permute_bf16");
    });
    m.def("dact_f32_bf16", [](uptr out, uptr in, uptr H, long n, uptr stream) {
        check(hpnn_dact_f32_bf16(P(out), (const float *)P(in), P(H), n, S(stream)), "dact_f32_bf16");
    });
    m.def("pack_bf16", [](uptr src, int src_f64, int rows, int cols, int lds, uptr dst, int prow, int pcol, int ldd,
                          uptr stream) {
        check(hpnn_pack_bf16(P(src), src_f64, rows, cols, lds, P(dst), prow, pcol, ldd, S(stream)), "pack_bf16");
    });
    m.def("fill_f32", [](uptr p, long n, float v, uptr stream) {
        check(hpnn_fill_f32((float *)P(p), n, v, S(stream)), "fill_f32");
    });
    m.def("mlp3_mid", [](uptr H1, uptr W1, uptr W1t, uptr W2, uptr W2t, uptr labels, uptr T, int ldt, float t_hi,
                         float t_lo, uptr D1, uptr gslab, uptr loss, uptr correct, int Bp, int n_valid, int n_out,
                         int type, int h1, int h2, int no, int grid, uptr stream) {
        check(hpnn_mlp3_mid(P(H1), P(W1), P(W1t), P(W2), P(W2t), (const int *)P(labels), (const float *)P(T), ldt,
                            t_hi, t_lo, P(D1), (float *)P(gslab), (float *)P(loss), (unsigned int *)P(correct), Bp,
                            n_valid, n_out, type, h1, h2, no, grid, S(stream)),
              "mlp3_mid");
    });
    m.def("reduce_slabs2", [](uptr slab, int Sn, long stride, long n, uptr tmp, uptr out, uptr stream) {
        check(hpnn_reduce_slabs2((const float *)P(slab), Sn, stride, n, (float *)P(tmp), (float *)P(out), S(stream)),
              "reduce_slabs2");
    });
    m.def("mlp3_slab_floats", []() { return hpnn_mlp3_slab_floats(); });
    m.def("mlp3_fused", [](uptr X, int ldx, int K0, uptr W0f, uptr W1, uptr W2, uptr labels, uptr T, int ldt,
                           float t_hi, float t_lo, uptr D1, uptr gslab, uptr loss, uptr correct, int Bp, int n_valid,
                           int n_out, int type, int grid, int d1fm, uptr stream) {
        const int rc = hpnn_mlp3_fused(P(X), ldx, K0, P(W0f), P(W1), P(W2), (const int *)P(labels),
                                       (const float *)P(T), ldt, t_hi, t_lo, P(D1), (float *)P(gslab), (float *)P(loss),
                                       (unsigned int *)P(correct), Bp, n_valid, n_out, type, grid, d1fm, S(stream));
        if (rc <= 0) check(rc ? rc : -1, "mlp3_fused");
        return rc;
    });
    m.def("mlp3_tile", [](uptr Xg, int xu8, float xscale, int K0, uptr W0f, uptr W1, uptr W2, uptr W2t, uptr labels,
                          uptr T, int ldt, float t_hi, float t_lo, uptr D1, uptr gslab, uptr loss, uptr correct, int Bp,
                          int n_valid, int n_out, int type, int grid, uptr stream) {
        const int rc = hpnn_mlp3_tile(P(Xg), xu8, xscale, K0, P(W0f), P(W1), P(W2), P(W2t), (const int *)P(labels),
                                      (const float *)P(T), ldt, t_hi, t_lo, P(D1), (float *)P(gslab), (float *)P(loss),
                                      (unsigned int *)P(correct), Bp, n_valid, n_out, type, grid, S(stream));
        if (rc <= 0) check(rc ? rc : -1, "mlp3_tile");
        return rc;
    });
    m.def("gemm_fp", [](int f64, uptr A, int lda, int ta, uptr B, int ldb, int tb, uptr C, int ldc, uptr aux, int ldaux,
                        int M, int N, int K, int epi, int splits, long slab_stride, uptr stream) {
        check(hpnn_gemm_fp(f64, P(A), lda, ta, P(B), ldb, tb, P(C), ldc, P(aux), ldaux, M, N, K, epi, splits,
                           slab_stride, S(stream)),
              "gemm_fp");
        return hpnn_gemm_fp_splits(K, splits);
    });
    m.def("output_fp", [](int f64, uptr Z, int ldz, uptr T, int ldt, uptr D, int ldd, uptr O, int ldo, uptr guess,
                          uptr loss, uptr correct, int B, int n_valid, int n_out, int type, uptr stream) {
        check(hpnn_output_fp(f64, P(Z), ldz, P(T), ldt, P(D), ldd, P(O), ldo, (int *)P(guess), (float *)P(loss),
                             (unsigned int *)P(correct), B, n_valid, n_out, type, S(stream)),
              "output_fp");
    });
    m.def("update_fp", [](int f64, uptr W, uptr V, uptr G, int Sn, long gstride, long n, double lr, double alpha,
                          double scale, int momentum, uptr stream) {
        check(hpnn_update_fp(f64, P(W), P(V), P(G), Sn, gstride, n, lr, alpha, scale, momentum, S(stream)),
              "update_fp");
    });
    m.def("wide2_front", [](uptr X, int ldx, int K0, uptr W0, uptr W1, uptr W1t, uptr labels, uptr T, int ldt,
                            float t_hi, float t_lo, uptr H0, uptr D2, uptr D1, uptr pbuf, uptr cnt, uptr flag, uptr err,
                            uptr loss, uptr correct, int Bp, int n_valid, int n_out, int type, int ksplit,
                            uptr stream) {
        hpnn_wide2_args a;
        a.X = P(X), a.W0 = P(W0), a.W1 = P(W1), a.W1t = P(W1t);
        a.ldx = ldx, a.K0 = K0;
        a.labels = (const int *)P(labels);
        a.T = (const float *)P(T);
        a.ldt = ldt, a.t_hi = t_hi, a.t_lo = t_lo;
        a.H0 = P(H0), a.D2 = P(D2), a.D1 = P(D1), a.pbuf = P(pbuf);
        a.cnt = (unsigned int *)P(cnt), a.flag = (unsigned int *)P(flag), a.err = (unsigned int *)P(err);
        a.loss_acc = (float *)P(loss), a.correct = (unsigned int *)P(correct);
        a.Bp = Bp, a.n_valid = n_valid, a.n_out = n_out, a.type = type, a.ksplit = ksplit;
        check(hpnn_wide2_front(&a, S(stream)), "wide2_front");
    });
    m.def("tn8_trace", []() {
        std::vector<unsigned long long> v(512 * 8);
        check(hpnn_tn8_trace(v.data()), "tn8_trace");
        return v;
    });
    m.def("wide2_ksplit", [](int Bp, int K0) { return hpnn_wide2_ksplit(Bp, K0); });
    m.def("wide2_pbuf_bytes", [](int Bp) { return hpnn_wide2_pbuf_bytes(Bp); });
    m.def("wide2_trace", []() {
        std::vector<unsigned long long> v(512 * 12);
        check(hpnn_wide2_trace(v.data()), "wide2_trace");
        return v;
    });
    m.def("mlp3_tile_grid", [](int Bp, int grid) { return hpnn_mlp3_tile_grid(Bp, grid); });
    m.def("mlp3_tile_trace", []() {
        std::vector<unsigned long long> v(1024 * 12);
        check(hpnn_mlp3_tile_trace(v.data()), "mlp3_tile_trace");
        return v;
    });
    m.def("g0_trace", []() {
        std::vector<unsigned long long> v(512 * 8);
        check(hpnn_g0_trace(v.data()), "g0_trace");
        return v;
    });
    m.def("mlp3_fused_grid", [](int Bp, int grid) { return hpnn_mlp3_fused_grid(Bp, grid); });
    m.def("gemm_fm_direct", [](uptr Dg, uptr Hg, int h_u8, float hscale, uptr slab, int ldg, int N, int M, int Bt,
                               int splits, uptr stream) {
        check(hpnn_gemm_fm_direct(P(Dg), P(Hg), h_u8, hscale, (float *)P(slab), ldg, N, M, Bt, splits, S(stream)),
              "gemm_fm_direct");
    });
    m.def("gemm_fm_direct_reduce", [](uptr Dg, uptr Hg, int h_u8, float hscale, uptr slab, int ldg, int N, int M,
                                      int Bt, int splits, uptr rslab, int rS, long rstride, long rn, int rgroups,
                                      uptr rout, uptr stream) {
        check(hpnn_gemm_fm_direct_reduce(P(Dg), P(Hg), h_u8, hscale, (float *)P(slab), ldg, N, M, Bt, splits,
                                         (const float *)P(rslab), rS, rstride, rn, rgroups, (float *)P(rout),
                                         S(stream)),
              "gemm_fm_direct_reduce");
    });
    m.def("gemm_tn_bf16_reduce", [](uptr D, int ldd, uptr H, int ldh, uptr slab, int ldg, int N, int M, int Bt,
                                    int splits, uptr rslab, int rS, long rstride, long rn, int rgroups, uptr rout,
                                    uptr stream) {
        check(hpnn_gemm_tn_bf16_reduce(P(D), ldd, P(H), ldh, (float *)P(slab), ldg, N, M, Bt, splits,
                                       (const float *)P(rslab), rS, rstride, rn, rgroups, (float *)P(rout), S(stream)),
              "gemm_tn_bf16_reduce");
    });
    m.def("reduce_groups", [](uptr slab, int Sn, long stride, long n, int groups, uptr out, uptr stream) {
        check(hpnn_reduce_groups((const float *)P(slab), Sn, stride, n, groups, (float *)P(out), S(stream)),
              "reduce_groups");
    });
    m.def(
        "sgd_update_multi",
        [](py::list layers, float lr, float alpha, float scale, int momentum, uptr stream) {
            hpnn_upd_layer L[HPNN_UPD_MAX];
            const int n = (int)py::len(layers);
            if (n < 1 || n > HPNN_UPD_MAX) throw std::runtime_error("sgd_update_multi: 1..8 layers");
            for (int i = 0; i < n; i++) {
                py::tuple t = layers[i].cast<py::tuple>();
                if (py::len(t) != 10) throw std::runtime_error("sgd_update_multi: layer tuple of 10");
                L[i].W32 = (float *)P(t[0].cast<uptr>());
                L[i].V32 = (float *)P(t[1].cast<uptr>());
                L[i].G = (const float *)P(t[2].cast<uptr>());
                L[i].gstride = t[3].cast<long>();
                L[i].Wbf = P(t[4].cast<uptr>());
                L[i].Wt = P(t[5].cast<uptr>());
                L[i].Wf = P(t[6].cast<uptr>());
                L[i].S = t[7].cast<int>();
                L[i].N = t[8].cast<int>();
                L[i].K = t[9].cast<int>();
            }
            check(hpnn_sgd_update_multi(L, n, lr, alpha, scale, momentum, S(stream)), "sgd_update_multi");
        },
        "layers: [(W32, V32, G, gstride, Wbf, Wt, Wf, S, N, K)] device addresses (0 = none)");
    /* ---- communication layer (include/libhpnn/comm.h) ---- */
    m.def("comm_available", []() { return hpnn_comm_available(); });
    m.def("comm_unique_id", []() {
        unsigned char id[HPNN_COMM_ID_BYTES];
        check(hpnn_comm_unique_id(id), "comm_unique_id");
        return py::bytes((const char *)id, HPNN_COMM_ID_BYTES);
    });
    m.def(
        "comm_init_rank",
        [](py::bytes id, int nranks, int rank, int device) {
            const std::string s = id;
            if (s.size() != HPNN_COMM_ID_BYTES) throw std::runtime_error("comm id must be 128 bytes");
            py::gil_scoped_release nogil; /* collective: blocks until every rank joined */
            return (uptr)hpnn_comm_init_rank((const unsigned char *)s.data(), nranks, rank, device);
        },
        "RCCL communicator of this process' device (0 on failure)");
    m.def("comm_destroy", [](uptr c) { hpnn_comm_destroy((hpnn_comm *)c); });
    m.def("comm_rank", [](uptr c) { return hpnn_comm_rank((const hpnn_comm *)c); });
    m.def("comm_size", [](uptr c) { return hpnn_comm_size((const hpnn_comm *)c); });
    m.def("comm_all_reduce", [](uptr c, uptr send, uptr recv, long count, int dt, int op, uptr stream) {
        check(hpnn_comm_all_reduce((hpnn_comm *)c, P(send), P(recv), count, (hpnn_comm_dtype)dt, (hpnn_comm_op)op,
                                   S(stream)),
              "comm_all_reduce");
    });
    m.def("comm_broadcast", [](uptr c, uptr send, uptr recv, long count, int dt, int root, uptr stream) {
        check(hpnn_comm_broadcast((hpnn_comm *)c, P(send), P(recv), count, (hpnn_comm_dtype)dt, root, S(stream)),
              "comm_broadcast");
    });
    m.def("comm_all_gather", [](uptr c, uptr send, uptr recv, long count, int dt, uptr stream) {
        check(hpnn_comm_all_gather((hpnn_comm *)c, P(send), P(recv), count, (hpnn_comm_dtype)dt, S(stream)),
              "comm_all_gather");
    });
    m.def("comm_reduce_scatter", [](uptr c, uptr send, uptr recv, long count, int dt, int op, uptr stream) {
        check(hpnn_comm_reduce_scatter((hpnn_comm *)c, P(send), P(recv), count, (hpnn_comm_dtype)dt,
                                       (hpnn_comm_op)op, S(stream)),
              "comm_reduce_scatter");
    });
    m.def("comm_all_reduce_async", [](uptr c, uptr buf, long count, int dt, uptr stream) {
        check(hpnn_comm_all_reduce_async((hpnn_comm *)c, P(buf), count, (hpnn_comm_dtype)dt, S(stream)),
              "comm_all_reduce_async");
    });
    m.def("comm_join", [](uptr c, uptr stream) { check(hpnn_comm_join((hpnn_comm *)c, S(stream)), "comm_join"); });
    m.def("comm_check", [](uptr c) { return hpnn_comm_check((hpnn_comm *)c); });
    m.def("comm_abort", [](uptr c) { hpnn_comm_abort((hpnn_comm *)c); });
    m.def("comm_all_ok", [](uptr c, int ok, uptr stream) {
        py::gil_scoped_release nogil;
        return hpnn_comm_all_ok((hpnn_comm *)c, ok, S(stream));
    });
    m.def("devmem_stats", []() {
        size_t a, b, c, d;
        hpnn_dev_stats(&a, &b, &c, &d);
        return py::make_tuple(a, b, c, d);
    });
    m.def("devmem_trim", []() { hpnn_dev_trim(); });
    m.def("fault_hit", [](const std::string &site) { return hpnn_fault_hit(site.c_str()); });
    /* one-shot xGMI all-reduce (include/libhpnn/xar.h) */
    m.attr("XAR_HANDLE_BYTES") = (int)HPNN_XAR_HANDLE_BYTES;
    m.def("xar_create", [](int rank, int world, size_t max_bytes) {
        return (uptr)hpnn_xar_create(rank, world, max_bytes);
    });
    m.def("xar_handles", [](uptr c) {
        std::string h(HPNN_XAR_HANDLE_BYTES, '\0');
        check(hpnn_xar_handles((hpnn_xar *)c, &h[0]), "xar_handles");
        return py::bytes(h);
    });
    m.def("xar_open", [](uptr c, py::bytes all) {
        std::string s = all;
        check(hpnn_xar_open((hpnn_xar *)c, s.data()), "xar_open");
    });
    m.def("xar_all_reduce_f32", [](uptr c, uptr in, uptr out, long count, uptr stream) {
        check(hpnn_xar_all_reduce_f32((hpnn_xar *)c, (const float *)P(in), (float *)P(out), count, S(stream)),
              "xar_all_reduce_f32");
    });
    m.def("xar_all_reduce_slabs_f32", [](uptr c, std::vector<std::tuple<uptr, long, int, long>> segs, uptr out,
                                         uptr stream) {
        std::vector<hpnn_xar_seg> v;
        for (auto &t : segs) v.push_back({(const float *)P(std::get<0>(t)), std::get<1>(t), std::get<2>(t), std::get<3>(t)});
        check(hpnn_xar_all_reduce_slabs_f32((hpnn_xar *)c, v.data(), (int)v.size(), (float *)P(out), S(stream)),
              "xar_all_reduce_slabs_f32");
    });
    m.def("xar_all_reduce_slabs_update_f32",
          [](uptr c, std::vector<std::tuple<uptr, long, int, long>> segs, uptr out,
             std::vector<std::tuple<uptr, uptr, uptr, uptr, uptr, int, int>> layers, float lr, float alpha, float scale,
             int momentum, uptr stream) {
              std::vector<hpnn_xar_seg> v;
              for (auto &t : segs)
                  v.push_back({(const float *)P(std::get<0>(t)), std::get<1>(t), std::get<2>(t), std::get<3>(t)});
              std::vector<hpnn_xar_upd_layer> L;
              for (auto &t : layers)
                  L.push_back({(float *)P(std::get<0>(t)), (float *)P(std::get<1>(t)), P(std::get<2>(t)),
                               P(std::get<3>(t)), P(std::get<4>(t)), std::get<5>(t), std::get<6>(t)});
              check(hpnn_xar_all_reduce_slabs_update_f32((hpnn_xar *)c, v.data(), (int)v.size(), (float *)P(out),
                                                         L.data(), (int)L.size(), lr, alpha, scale, momentum,
                                                         S(stream)),
                    "xar_all_reduce_slabs_update_f32");
          });
    m.def("xar_local", [](uptr c) {
        float *buf = nullptr;
        long half = 0;
        const unsigned int *sel = nullptr;
        check(hpnn_xar_local((hpnn_xar *)c, &buf, &half, &sel), "xar_local");
        return py::make_tuple((uptr)buf, (uptr)sel, half);
    });
    m.def("xar_reduce_local_update_f32",
          [](uptr c, long count, uptr out, std::vector<std::tuple<uptr, uptr, uptr, uptr, uptr, int, int>> layers,
             float lr, float alpha, float scale, int momentum, uptr stream) {
              std::vector<hpnn_xar_upd_layer> L;
              for (auto &t : layers)
                  L.push_back({(float *)P(std::get<0>(t)), (float *)P(std::get<1>(t)), P(std::get<2>(t)),
                               P(std::get<3>(t)), P(std::get<4>(t)), std::get<5>(t), std::get<6>(t)});
              check(hpnn_xar_reduce_local_update_f32((hpnn_xar *)c, count, (float *)P(out), L.data(), (int)L.size(), lr,
                                                     alpha, scale, momentum, S(stream)),
                    "xar_reduce_local_update_f32");
          });
    m.def("xar_status", [](uptr c) { return hpnn_xar_status((hpnn_xar *)c); });
    m.def("xar_self_test", [](uptr c, uptr stream) { return hpnn_xar_self_test((hpnn_xar *)c, S(stream)); });
    m.def("xar_destroy", [](uptr c) { hpnn_xar_destroy((hpnn_xar *)c); });
    m.def("comm_set_xar", [](uptr c, uptr x, size_t max_bytes) {
        check(hpnn_comm_set_xar((hpnn_comm *)c, (hpnn_xar *)x, max_bytes), "comm_set_xar");
    });
    m.def("device_count", []() {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        return n;
    });
}
