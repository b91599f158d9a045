// pybind11 surface of the mxddp native extension.  Device buffers cross the boundary as
// raw addresses (ints) and streams as hipStream_t handles, so this TU never includes
// torch headers: the Python layer (mxddp/ops) owns tensors, validates shapes / dtypes /
// devices, and passes `tensor.data_ptr()` and `torch.cuda.current_stream().cuda_stream`.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "comm.h"
#include "common.h"
#include "keras_engine.h"
#include "mlp_engine.h"
#include "mnist_engine.h"
#include "ops.h"
#include "peer.h"
#include "reducer.h"
#include "wgrad_defer.h"

namespace py = pybind11;
using namespace mx;

namespace {
template <class T>
T* P(uintptr_t v) { return reinterpret_cast<T*>(v); }
hipStream_t S(uintptr_t v) { return reinterpret_cast<hipStream_t>(v); }
ConvShape CS(int N, int C, int H, int W, int K, int R, int S_, int sh, int sw, int ph, int pw, int dh, int dw) {
  return ConvShape::make(N, C, H, W, K, R, S_, sh, sw, ph, pw, dh, dw);
}
}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "mxddp native kernels (gfx950), RCCL communicator, reducer and fused engines";
  m.attr("ARCH") = "gfx950";

  // ---------------------------------------------------------------- GEMM-shaped ops
  m.def("conv2d_fwd", [](uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t y, int N, int C, int H, int W, int K, int R,
                         int S_, int sh, int sw, int ph, int pw, int dh, int dw, bool relu, uintptr_t st,
                         uintptr_t scratch, uintptr_t dgrad_filters, bool pretransformed, uintptr_t in_ss,
                         bool in_relu) {
    conv2d_fwd(P<const float>(x), P<const float>(w), P<const float>(b), P<float>(y),
               CS(N, C, H, W, K, R, S_, sh, sw, ph, pw, dh, dw), relu, S(st), P<float>(scratch),
               P<float>(dgrad_filters), pretransformed, P<const float>(in_ss), in_relu);
  }, py::arg("x"), py::arg("w"), py::arg("b"), py::arg("y"), py::arg("N"), py::arg("C"), py::arg("H"), py::arg("W"),
     py::arg("K"), py::arg("R"), py::arg("S"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"),
     py::arg("dh"), py::arg("dw"), py::arg("relu"), py::arg("st"), py::arg("scratch") = 0,
     py::arg("dgrad_filters") = 0, py::arg("pretransformed") = false, py::arg("in_ss") = 0,
     py::arg("in_relu") = false);
  m.def("conv_fwd_filter_floats", [](int N, int C, int H, int W, int K, int R, int S_, int sh, int sw, int ph,
                                     int pw, int dh, int dw) {
    return conv_fwd_filter_floats(CS(N, C, H, W, K, R, S_, sh, sw, ph, pw, dh, dw));
  });
  py::class_<WinoFilterBank>(m, "WinoFilterBank", "persistent Winograd filters of many convs, one refresh launch")
      .def(py::init<>())
      .def("add", [](WinoFilterBank& b, uintptr_t w, uintptr_t uf, uintptr_t ud, int K, int C) {
        b.add(P<const float>(w), P<float>(uf), P<float>(ud), K, C);
      })
      .def("clear", &WinoFilterBank::clear)
      .def("size", &WinoFilterBank::size)
      .def("refresh", [](const WinoFilterBank& b, uintptr_t st) { b.refresh(S(st)); });
  m.def("conv_dgrad_filter_floats", [](int N, int C, int H, int W, int K, int R, int S_, int sh, int sw, int ph,
                                       int pw, int dh, int dw) {
    return conv_dgrad_filter_floats(CS(N, C, H, W, K, R, S_, sh, sw, ph, pw, dh, dw));
  });
  m.def("conv_scratch_floats", [](int N, int C, int H, int W, int K, int R, int S_, int sh, int sw, int ph, int pw,
                                  int dh, int dw) {
    return conv_scratch_floats(CS(N, C, H, W, K, R, S_, sh, sw, ph, pw, dh, dw));
  });
  m.def("set_conv_algo", &set_conv_algo, "3x3 s1 convs: 0 = auto (Winograd F(2x2,3x3) where eligible), 1 = direct");
  m.def("conv_algo", &conv_algo);
  m.def("conv2d_dgrad", [](uintptr_t dy, uintptr_t w, uintptr_t dx, int N, int C, int H, int W, int K, int R, int S_,
                           int sh, int sw, int ph, int pw, int dh, int dw, uintptr_t mask, bool acc, uintptr_t st,
                           uintptr_t wt_scratch, bool pretransformed) {
    conv2d_dgrad(P<const float>(dy), P<const float>(w), P<float>(dx), CS(N, C, H, W, K, R, S_, sh, sw, ph, pw, dh, dw),
                 P<const float>(mask), acc, S(st), P<float>(wt_scratch), pretransformed);
  }, py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("N"), py::arg("C"), py::arg("H"), py::arg("W"), py::arg("K"),
     py::arg("R"), py::arg("S"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("dh"),
     py::arg("dw"), py::arg("mask"), py::arg("acc"), py::arg("st"), py::arg("wt_scratch") = 0,
     py::arg("pretransformed") = false);
  m.def("conv2d_wgrad", [](uintptr_t dy, uintptr_t x, uintptr_t dw_, int N, int C, int H, int W, int K, int R, int S_,
                           int sh, int sw, int ph, int pw, int dh, int dw, bool acc, uintptr_t st,
                           uintptr_t scratch, uintptr_t db, uintptr_t in_ss, bool in_relu) {
    return conv2d_wgrad(P<const float>(dy), P<const float>(x), P<float>(dw_),
                        CS(N, C, H, W, K, R, S_, sh, sw, ph, pw, dh, dw), acc, S(st), P<float>(scratch), P<float>(db),
                        P<const float>(in_ss), in_relu);
  }, py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("N"), py::arg("C"), py::arg("H"), py::arg("W"), py::arg("K"),
     py::arg("R"), py::arg("S"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("dh"),
     py::arg("dwd"), py::arg("acc"), py::arg("st"), py::arg("scratch") = 0, py::arg("db") = 0, py::arg("in_ss") = 0,
     py::arg("in_relu") = false);
  m.def("conv_wgrad_scratch_floats", [](int N, int C, int H, int W, int K, int R, int S_, int sh, int sw, int ph,
                                        int pw, int dh, int dw) {
    return conv_wgrad_scratch_floats(CS(N, C, H, W, K, R, S_, sh, sw, ph, pw, dh, dw));
  });
  m.def("linear_fwd", [](uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t y, int M, int N, int K, bool relu,
                         uintptr_t st) {
    linear_fwd(P<const float>(x), P<const float>(w), P<const float>(b), P<float>(y), M, N, K, relu, S(st));
  });
  m.def("linear_dgrad", [](uintptr_t dy, uintptr_t w, uintptr_t dx, int M, int N, int K, uintptr_t mask, bool acc,
                           uintptr_t st, uintptr_t dy_mask) {
    linear_dgrad(P<const float>(dy), P<const float>(w), P<float>(dx), M, N, K, P<const float>(mask), acc, S(st),
                 P<const float>(dy_mask));
  }, py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("mask"),
     py::arg("acc"), py::arg("st"), py::arg("dy_mask") = 0);
  m.def("linear_wgrad", [](uintptr_t dy, uintptr_t x, uintptr_t dw, int M, int N, int K, bool acc, uintptr_t st,
                           uintptr_t dy_mask) {
    linear_wgrad(P<const float>(dy), P<const float>(x), P<float>(dw), M, N, K, acc, S(st), P<const float>(dy_mask));
  }, py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("acc"),
     py::arg("st"), py::arg("dy_mask") = 0);

  // ---------------------------------------------------------------- channels-last bf16 (nhwc_bf16.hip)
  m.def("nhwc_from_nchw", [](uintptr_t x, uintptr_t y, int N, int C, int H, int W, int Cp, uintptr_t st) {
    nhwc_from_nchw(P<const float>(x), P<uint16_t>(y), N, C, H, W, Cp, S(st));
  });
  m.def("nhwc_repack_weight", [](uintptr_t w, uintptr_t wt, uintptr_t wtd, int K, int C, int R, int S_, int Cp,
                                 uintptr_t st) {
    nhwc_repack_weight(P<const float>(w), P<uint16_t>(wt), P<uint16_t>(wtd), K, C, R, S_, Cp, S(st));
  });
  m.def("nhwc_repack_blocks", &nhwc_repack_blocks);
  m.def("nhwc_conv_bn_rows", &nhwc_conv_bn_rows);
  m.def("nhwc_conv_dgrad_scratch_floats", &nhwc_conv_dgrad_scratch_floats);
  m.def("nhwc_conv_set_glds", &nhwc_conv_set_glds);
  m.def("nhwc_conv_set_glds256", &nhwc_conv_set_glds256);
  m.def("nhwc_conv_set_glds_short", &nhwc_conv_set_glds_short);
  m.def("nhwc_conv_set_glds_deep", &nhwc_conv_set_glds_deep);
  m.def("nhwc_conv_set_glds_par", &nhwc_conv_set_glds_par);
  m.def("nhwc_conv_set_gk2", &nhwc_conv_set_gk2);
  m.def("nhwc_wgrad_set_waves8", &nhwc_wgrad_set_waves8);
  m.def("nhwc_bn_set_grid_cap", &nhwc_bn_set_grid_cap);
  m.def("nhwc_bn_set_wt", &nhwc_bn_set_wt);
  m.def("nhwc_conv_set_wt", &nhwc_conv_set_wt);
  m.def("nhwc_conv_set_split_blocks", &nhwc_conv_set_split_blocks);
  m.def("nhwc_wgrad_set_target", &nhwc_wgrad_set_target);
  m.def("nhwc_wgrad_set_small_npix", &nhwc_wgrad_set_small_npix);
  m.def("wino_wgrad_set_slots", &wino_wgrad_set_slots);
  m.def("nhwc_wgrad_set_tile256", &nhwc_wgrad_set_tile256);
  m.def("wgrad_defer_set", &wgrad_defer_set,
        "this thread's next weight-gradient calls record their split reduction for wgrad_defer_flush");
  m.def("wgrad_defer_took", &wgrad_defer_took);
  m.def("wgrad_defer_pending", &wgrad_defer_pending);
  m.def("wgrad_defer_flush", [](uintptr_t st) { return wgrad_defer_flush(S(st)); });
  m.def("mnist_set_fc1_defer", &mnist_set_fc1_defer,
        "fused MNIST, world size 1: fc1 weight gradient + SGD in the conv-backward launch's last blocks (1) or in F5 (0)");
  m.def("mnist_fc1_defer", &mnist_fc1_defer);
  m.def("mnist_set_f67_order", &mnist_set_f67_order,
        "fused MNIST batch 64: XCD-aware placement of the conv-backward launch's blocks (1) or plain order (0)");
  m.def("mnist_f67_order", &mnist_f67_order);
  m.def("mlp_set_w2_defer", &mlp_set_w2_defer,
        "fused MLP: the dW2 tile + update as extra resident blocks of K5 (1) or in K4 (0, default)");
  m.def("mlp_w2_defer", &mlp_w2_defer);
  m.def("mnist_set_wt_stores", &mnist_set_wt_stores,
        "MNIST bulk stores with agent scope (L2 write-through) for steps launched afterwards: mask 1 = F5, 2 = F2, "
        "4 = F6W");
  m.def("mnist_wt_stores", &mnist_wt_stores);
  m.def("nhwc_repack_many", [](uintptr_t desc, int n, int total_blocks, uintptr_t st) {
    nhwc_repack_many(P<const int64_t>(desc), n, total_blocks, S(st));
  });
  m.def("nhwc_conv_fwd", [](uintptr_t x, uintptr_t wt, uintptr_t y, int N, int H, int W, int Cp, int K, int R, int S_,
                            int sh, int sw, int ph, int pw, int P_, int Q, uintptr_t scratch, uintptr_t st,
                            uintptr_t bnpart, uintptr_t bnshift) {
    return nhwc_conv_fwd(P<const uint16_t>(x), P<const uint16_t>(wt), P<uint16_t>(y), N, H, W, Cp, K, R, S_, sh, sw,
                         ph, pw, P_, Q, P<float>(scratch), S(st), P<float>(bnpart), P<const float>(bnshift));
  }, py::arg("x"), py::arg("wt"), py::arg("y"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("Cp"), py::arg("K"),
     py::arg("R"), py::arg("S"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("P"), py::arg("Q"),
     py::arg("scratch"), py::arg("st"), py::arg("bnpart") = 0, py::arg("bnshift") = 0);
  m.def("nhwc_conv_scratch_floats", &nhwc_conv_scratch_floats);
  m.def("nhwc_conv_dgrad", [](uintptr_t dy, uintptr_t wt, uintptr_t dx, int N, int H, int W, int C, int K, int R,
                              int S_, int sh, int sw, int ph, int pw, int P_, int Q, uintptr_t scratch,
                              uintptr_t st, uintptr_t addend, uintptr_t bnpart, uintptr_t bx, uintptr_t bmean,
                              uintptr_t bfcoef, uintptr_t bmask, bool brelu, uintptr_t amask, bool addend_sub) {
    return nhwc_conv_dgrad(P<const uint16_t>(dy), P<const uint16_t>(wt), P<uint16_t>(dx), N, H, W, C, K, R, S_, sh, sw,
                           ph, pw, P_, Q, P<float>(scratch), S(st), P<const uint16_t>(addend), P<float>(bnpart),
                           P<const uint16_t>(bx), P<const float>(bmean), P<const float>(bfcoef),
                           P<const uint8_t>(bmask), brelu, P<const uint8_t>(amask), addend_sub);
  }, py::arg("dy"), py::arg("wt"), py::arg("dx"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("K"),
     py::arg("R"), py::arg("S"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("P"), py::arg("Q"),
     py::arg("scratch"), py::arg("st"), py::arg("addend") = 0, py::arg("bnpart") = 0, py::arg("bx") = 0,
     py::arg("bmean") = 0, py::arg("bfcoef") = 0, py::arg("bmask") = 0, py::arg("brelu") = false,
     py::arg("amask") = 0, py::arg("addend_sub") = false);
  m.def("nhwc_conv_dgrad_bn_rows", &nhwc_conv_dgrad_bn_rows);
  m.def("nhwc_conv_wgrad", [](uintptr_t dy, uintptr_t x, uintptr_t dw, int N, int H, int W, int Cin, int Cp, int K,
                              int R, int S_, int sh, int sw, int ph, int pw, int P_, int Q, bool acc, uintptr_t scratch,
                              uintptr_t st) {
    nhwc_conv_wgrad(P<const uint16_t>(dy), P<const uint16_t>(x), P<float>(dw), N, H, W, Cin, Cp, K, R, S_, sh, sw, ph,
                    pw, P_, Q, acc, P<float>(scratch), S(st));
  });
  m.def("nhwc_wgrad_scratch_floats", &nhwc_wgrad_scratch_floats);
  m.def("nhwc_bn_fwd", [](uintptr_t x, uintptr_t res, uintptr_t y, uintptr_t g, uintptr_t b, uintptr_t mean,
                          uintptr_t invstd, uintptr_t rm, uintptr_t rv, uintptr_t nbt, int Npix, int C, float mom,
                          float eps, bool relu, uintptr_t scratch, uintptr_t st, uintptr_t coef_out,
                          uintptr_t mask_out, uintptr_t pre_part, int pre_gx, uintptr_t kshift) {
    nhwc_bn_fwd(P<const uint16_t>(x), P<const uint16_t>(res), P<uint16_t>(y), P<const float>(g), P<const float>(b),
                P<float>(mean), P<float>(invstd), P<float>(rm), P<float>(rv), P<int64_t>(nbt), Npix, C, mom, eps, relu,
                P<float>(scratch), S(st), P<float>(coef_out), P<uint8_t>(mask_out), P<const float>(pre_part), pre_gx,
                P<const float>(kshift));
  }, py::arg("x"), py::arg("res"), py::arg("y"), py::arg("g"), py::arg("b"), py::arg("mean"), py::arg("invstd"),
     py::arg("rm"), py::arg("rv"), py::arg("nbt"), py::arg("Npix"), py::arg("C"), py::arg("mom"), py::arg("eps"),
     py::arg("relu"), py::arg("scratch"), py::arg("st"), py::arg("coef_out") = 0, py::arg("mask_out") = 0,
     py::arg("pre_part") = 0, py::arg("pre_gx") = 0, py::arg("kshift") = 0);
  m.def("nhwc_bn_scratch_floats", &nhwc_bn_scratch_floats);
  m.def("nhwc_bn_bwd", [](uintptr_t dy, uintptr_t x, uintptr_t y, uintptr_t g, uintptr_t mean, uintptr_t invstd,
                          uintptr_t dx, uintptr_t dres, uintptr_t dg, uintptr_t db, int Npix, int C, bool relu,
                          bool accp, uintptr_t scratch, uintptr_t st, uintptr_t fcoef, uintptr_t mask,
                          uintptr_t pre_part, int pre_gx) {
    nhwc_bn_bwd(P<const uint16_t>(dy), P<const uint16_t>(x), P<const uint16_t>(y), P<const float>(g),
                P<const float>(mean), P<const float>(invstd), P<uint16_t>(dx), P<uint16_t>(dres), P<float>(dg),
                P<float>(db), Npix, C, relu, accp, P<float>(scratch), S(st), P<const float>(fcoef),
                P<const uint8_t>(mask), P<const float>(pre_part), pre_gx);
  }, py::arg("dy"), py::arg("x"), py::arg("y"), py::arg("g"), py::arg("mean"), py::arg("invstd"), py::arg("dx"),
     py::arg("dres"), py::arg("dg"), py::arg("db"), py::arg("Npix"), py::arg("C"), py::arg("relu"), py::arg("accp"),
     py::arg("scratch"), py::arg("st"), py::arg("fcoef") = 0, py::arg("mask") = 0, py::arg("pre_part") = 0,
     py::arg("pre_gx") = 0);
  m.def("nhwc_maxpool_fwd", [](uintptr_t x, uintptr_t y, uintptr_t arg, int N, int H, int W, int C, int P_, int Q,
                               int k, int s, int p, uintptr_t st) {
    nhwc_maxpool_fwd(P<const uint16_t>(x), P<uint16_t>(y), P<uint8_t>(arg), N, H, W, C, P_, Q, k, s, p, S(st));
  });
  m.def("nhwc_maxpool_bwd", [](uintptr_t dy, uintptr_t arg, uintptr_t dx, int N, int H, int W, int C, int P_, int Q,
                               int k, int s, int p, uintptr_t st) {
    nhwc_maxpool_bwd(P<const uint16_t>(dy), P<const uint8_t>(arg), P<uint16_t>(dx), N, H, W, C, P_, Q, k, s, p, S(st));
  });
  m.def("nhwc_gap_fwd", [](uintptr_t x, uintptr_t y, int N, int HW, int C, uintptr_t st) {
    nhwc_gap_fwd(P<const uint16_t>(x), P<float>(y), N, HW, C, S(st));
  });
  m.def("nhwc_gap_bwd", [](uintptr_t dy, uintptr_t dx, int N, int HW, int C, uintptr_t st) {
    nhwc_gap_bwd(P<const float>(dy), P<uint16_t>(dx), N, HW, C, S(st));
  });

  m.def("set_gemm_precision", &set_gemm_precision);
  m.def("set_debug_sync", &set_debug_sync, "synchronise + check after every kernel launch (debugging)");
  m.def("debug_sync", &debug_sync);
  m.def("gemm_precision", &gemm_precision);

  // ---------------------------------------------------------------- elementwise
  m.def("relu_fwd", [](uintptr_t x, uintptr_t y, int64_t n, uintptr_t st) { relu_fwd(P<const float>(x), P<float>(y), n, S(st)); });
  m.def("relu_bwd", [](uintptr_t dy, uintptr_t y, uintptr_t dx, int64_t n, uintptr_t st) {
    relu_bwd(P<const float>(dy), P<const float>(y), P<float>(dx), n, S(st));
  });
  m.def("bias_grad", [](uintptr_t dy, uintptr_t db, int outer, int C, int inner, bool acc, uintptr_t st,
                        uintptr_t dy_mask) {
    bias_grad(P<const float>(dy), P<float>(db), outer, C, inner, acc, S(st), P<const float>(dy_mask));
  }, py::arg("dy"), py::arg("db"), py::arg("outer"), py::arg("C"), py::arg("inner"), py::arg("acc"), py::arg("st"),
     py::arg("dy_mask") = 0);
  m.def("add_inplace", [](uintptr_t y, uintptr_t x, int64_t n, uintptr_t st) { add_inplace(P<float>(y), P<const float>(x), n, S(st)); });
  m.def("scale_inplace", [](uintptr_t y, float a, int64_t n, uintptr_t st) { scale_inplace(P<float>(y), a, n, S(st)); });
  m.def("fill", [](uintptr_t y, float v, int64_t n, uintptr_t st) { fill(P<float>(y), v, n, S(st)); });
  m.def("maxpool2d_fwd", [](uintptr_t x, uintptr_t y, uintptr_t idx, int N, int C, int H, int W, int kh, int kw, int sh,
                            int sw, int ph, int pw, int P_, int Q, uintptr_t st) {
    maxpool2d_fwd(P<const float>(x), P<float>(y), P<int32_t>(idx), N, C, H, W, kh, kw, sh, sw, ph, pw, P_, Q, S(st));
  });
  m.def("maxpool2d_bwd", [](uintptr_t dy, uintptr_t idx, uintptr_t dx, int N, int C, int H, int W, int P_, int Q,
                            uintptr_t st, int sh, int sw) {
    maxpool2d_bwd(P<const float>(dy), P<const int32_t>(idx), P<float>(dx), N, C, H, W, P_, Q, S(st), sh, sw);
  }, py::arg("dy"), py::arg("idx"), py::arg("dx"), py::arg("N"), py::arg("C"), py::arg("H"), py::arg("W"),
     py::arg("P"), py::arg("Q"), py::arg("st"), py::arg("sh") = 0, py::arg("sw") = 0);
  m.def("avgpool2d_fwd", [](uintptr_t x, uintptr_t y, int N, int C, int H, int W, int kh, int kw, int sh, int sw, int ph,
                            int pw, int P_, int Q, uintptr_t st) {
    avgpool2d_fwd(P<const float>(x), P<float>(y), N, C, H, W, kh, kw, sh, sw, ph, pw, P_, Q, S(st));
  });
  m.def("avgpool2d_bwd", [](uintptr_t dy, uintptr_t dx, int N, int C, int H, int W, int kh, int kw, int sh, int sw,
                            int ph, int pw, int P_, int Q, uintptr_t st) {
    avgpool2d_bwd(P<const float>(dy), P<float>(dx), N, C, H, W, kh, kw, sh, sw, ph, pw, P_, Q, S(st));
  });
  m.def("xent_fwd_bwd", [](uintptr_t logits, uintptr_t y, uintptr_t logp, uintptr_t dlogits, uintptr_t loss_sum,
                           uintptr_t correct, int B, int C, float scale, uintptr_t st, float loss_scale) {
    xent_fwd_bwd(P<const float>(logits), P<const int32_t>(y), P<float>(logp), P<float>(dlogits), P<float>(loss_sum),
                 P<float>(correct), B, C, scale, S(st), loss_scale);
  }, py::arg("logits"), py::arg("y"), py::arg("logp"), py::arg("dlogits"), py::arg("loss_sum"), py::arg("correct"),
     py::arg("B"), py::arg("C"), py::arg("scale"), py::arg("st"), py::arg("loss_scale") = 1.f);
  m.def("bn_splits", &bn_splits);
  m.def("bn_fwd_train", [](uintptr_t x, uintptr_t g, uintptr_t b, uintptr_t y, uintptr_t mean, uintptr_t invstd,
                           uintptr_t rm, uintptr_t rv, int N, int C, int HW, float mom, float eps, bool relu,
                           uintptr_t part, uintptr_t st, uintptr_t nbt, uintptr_t res, int res_C, uintptr_t ss) {
    bn_fwd_train(P<const float>(x), P<const float>(g), P<const float>(b), P<float>(y), P<float>(mean), P<float>(invstd),
                 P<float>(rm), P<float>(rv), N, C, HW, mom, eps, relu, P<float>(part), S(st), P<int64_t>(nbt),
                 P<const float>(res), res_C, P<float>(ss));
  }, py::arg("x"), py::arg("g"), py::arg("b"), py::arg("y"), py::arg("mean"), py::arg("invstd"), py::arg("rm"),
     py::arg("rv"), py::arg("N"), py::arg("C"), py::arg("HW"), py::arg("mom"), py::arg("eps"), py::arg("relu"),
     py::arg("part"), py::arg("st"), py::arg("num_batches") = 0, py::arg("residual") = 0, py::arg("residual_C") = 0,
     py::arg("ss") = 0);
  m.def("bn_partial_floats", &bn_partial_floats);
  m.def("bn_fwd_eval", [](uintptr_t x, uintptr_t g, uintptr_t b, uintptr_t y, uintptr_t rm, uintptr_t rv, int N, int C,
                          int HW, float eps, bool relu, uintptr_t st) {
    bn_fwd_eval(P<const float>(x), P<const float>(g), P<const float>(b), P<float>(y), P<const float>(rm),
                P<const float>(rv), N, C, HW, eps, relu, S(st));
  });
  m.def("bn_bwd", [](uintptr_t dy, uintptr_t x, uintptr_t yr, uintptr_t g, uintptr_t mean, uintptr_t invstd,
                     uintptr_t dx, uintptr_t dg, uintptr_t db, int N, int C, int HW, bool acc, uintptr_t part,
                     uintptr_t st, uintptr_t extra, int extra_C, uintptr_t ssm) {
    bn_bwd(P<const float>(dy), P<const float>(x), P<const float>(yr), P<const float>(g), P<const float>(mean),
           P<const float>(invstd), P<float>(dx), P<float>(dg), P<float>(db), N, C, HW, acc, P<float>(part), S(st),
           P<const float>(extra), extra_C, P<const float>(ssm));
  }, py::arg("dy"), py::arg("x"), py::arg("yr"), py::arg("g"), py::arg("mean"), py::arg("invstd"), py::arg("dx"),
     py::arg("dg"), py::arg("db"), py::arg("N"), py::arg("C"), py::arg("HW"), py::arg("acc"), py::arg("part"),
     py::arg("st"), py::arg("extra") = 0, py::arg("extra_C") = 0, py::arg("ssm") = 0);
  m.def("shortcut_pad_add", [](uintptr_t x, uintptr_t y, int N, int Cin, int H, int W, int Cout, int P_, int Q,
                               int stride, uintptr_t st) {
    shortcut_pad_add(P<const float>(x), P<float>(y), N, Cin, H, W, Cout, P_, Q, stride, S(st));
  });
  m.def("shortcut_pad_add_bwd", [](uintptr_t dy, uintptr_t dx, int N, int Cin, int H, int W, int Cout, int P_, int Q,
                                   int stride, bool acc, uintptr_t st) {
    shortcut_pad_add_bwd(P<const float>(dy), P<float>(dx), N, Cin, H, W, Cout, P_, Q, stride, acc, S(st));
  });

  m.def("reserve_splitk_planes", [](uintptr_t st) { reserve_splitk_planes(S(st)); });

  // ---------------------------------------------------------------- optim / data
  m.def("sgd_step", [](uintptr_t p, uintptr_t g, uintptr_t buf, uintptr_t lr, float gscale, float mom, float wd,
                       int64_t n, bool first, uintptr_t st) {
    sgd_step(P<float>(p), P<const float>(g), P<float>(buf), P<const float>(lr), gscale, mom, wd, n, first, S(st));
  });
  m.def("adam_step", [](uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v, uintptr_t lr, uintptr_t state,
                        float gscale, float b1, float b2, float eps, float wd, bool eps_hat, int64_t n, uintptr_t st) {
    adam_step(P<float>(p), P<const float>(g), P<float>(mm), P<float>(v), P<const float>(lr), P<int32_t>(state),
              gscale, b1, b2, eps, wd, eps_hat, n, S(st));
  });
  m.def("synth_templates", [](uintptr_t t, int C, int D, uint64_t seed, uintptr_t st) {
    synth_templates(P<float>(t), C, D, seed, S(st));
  });
  m.def("synth_batch", [](uintptr_t x, uintptr_t y, uintptr_t t, int B, int D, int C, uint64_t seed, uintptr_t ctr,
                          uintptr_t st) {
    synth_batch(P<float>(x), P<int32_t>(y), P<const float>(t), B, D, C, seed, P<int32_t>(ctr), S(st));
  });
  m.def("augment_crop_flip_norm", [](uintptr_t x, uintptr_t y, int N, int C, int H, int W, int pad, uintptr_t mean,
                                     uintptr_t stdv, uint64_t seed, uintptr_t ctr, uintptr_t st) {
    augment_crop_flip_norm(P<const float>(x), P<float>(y), N, C, H, W, pad, P<const float>(mean), P<const float>(stdv),
                           seed, P<int32_t>(ctr), S(st));
  });
  m.def("count_correct", [](uintptr_t logits, uintptr_t y, uintptr_t correct, int B, int C, uintptr_t st) {
    count_correct(P<const float>(logits), P<const int32_t>(y), P<float>(correct), B, C, S(st));
  });

  // ---------------------------------------------------------------- communication
  py::enum_<DType>(m, "DType")
      .value("f32", DType::kF32).value("bf16", DType::kBF16).value("f16", DType::kF16)
      .value("i32", DType::kI32).value("i64", DType::kI64).value("u8", DType::kU8);
  py::enum_<RedOp>(m, "RedOp")
      .value("sum", RedOp::kSum).value("avg", RedOp::kAvg).value("max", RedOp::kMax)
      .value("min", RedOp::kMin).value("prod", RedOp::kProd);
  py::class_<Comm>(m, "Comm")
      .def(py::init([](py::bytes uid, int rank, int ws, int dev, int ctas, const std::string& algo,
                       const std::string& proto) {
             CommConfig cfg;
             cfg.ctas = ctas;
             cfg.algo = algo;
             cfg.proto = proto;
             std::string u(uid);
             py::gil_scoped_release nogil;  // the init waits for the other ranks
             return new Comm(u, rank, ws, dev, cfg);
           }),
           py::arg("uid"), py::arg("rank"), py::arg("world_size"), py::arg("device"), py::arg("ctas") = 0,
           py::arg("algo") = "", py::arg("proto") = "")
      .def_static("version", &Comm::version)
      .def_static("set_init_timeout", &Comm::set_init_timeout)
      .def_static("init_timeout", &Comm::init_timeout)
      .def_readonly_static("INIT_TIMEOUT_EXIT", &Comm::kInitTimeoutExit)
      .def_property_readonly("nranks", &Comm::nranks)
      .def_property_readonly("hip_device", &Comm::hip_device)
      .def_property_readonly("ctas", [](const Comm& c) { return c.config().ctas; })
      .def_property_readonly("variant", [](const Comm& c) { return c.config().name(); })
      .def_static("new_unique_id", []() { return py::bytes(Comm::new_unique_id()); })
      .def_static("init_all", [](const std::vector<int>& devs) {
        auto v = Comm::init_all(devs);
        py::list out;
        for (auto* c : v) out.append(py::cast(c, py::return_value_policy::take_ownership));
        return out;
      })
      .def("all_reduce", [](Comm& c, uintptr_t s, uintptr_t r, size_t n, DType t, RedOp o, uintptr_t st) {
        c.all_reduce(P<const void>(s), P<void>(r), n, t, o, S(st));
      })
      .def("broadcast", [](Comm& c, uintptr_t s, uintptr_t r, size_t n, DType t, int root, uintptr_t st) {
        c.broadcast(P<const void>(s), P<void>(r), n, t, root, S(st));
      })
      .def("reduce_scatter", [](Comm& c, uintptr_t s, uintptr_t r, size_t n, DType t, RedOp o, uintptr_t st) {
        c.reduce_scatter(P<const void>(s), P<void>(r), n, t, o, S(st));
      })
      .def("all_gather", [](Comm& c, uintptr_t s, uintptr_t r, size_t n, DType t, uintptr_t st) {
        c.all_gather(P<const void>(s), P<void>(r), n, t, S(st));
      })
      .def("all_to_all", [](Comm& c, uintptr_t s, uintptr_t r, size_t n, DType t, uintptr_t st) {
        c.all_to_all(P<const void>(s), P<void>(r), n, t, S(st));
      })
      .def("send", [](Comm& c, uintptr_t b, size_t n, DType t, int peer, uintptr_t st) { c.send(P<const void>(b), n, t, peer, S(st)); })
      .def("recv", [](Comm& c, uintptr_t b, size_t n, DType t, int peer, uintptr_t st) { c.recv(P<void>(b), n, t, peer, S(st)); })
      .def("check_async_error", &Comm::check_async_error)
      .def("abort", &Comm::abort)
      .def_static("group_start", &Comm::group_start)
      .def_static("group_end", &Comm::group_end)
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("world_size", &Comm::world_size)
      .def_property_readonly("device", &Comm::device);

  py::class_<PeerComm>(m, "PeerComm")
      .def(py::init<int, int, int, size_t, int>(), py::arg("rank"), py::arg("world_size"), py::arg("device"),
           py::arg("cap_bytes") = size_t(32) << 20, py::arg("blocks") = 64)
      .def("handles", [](const PeerComm& p) { return py::bytes(p.handles()); })
      .def("open", [](PeerComm& p, const std::vector<py::bytes>& all) {
        std::vector<std::string> v;
        for (auto& b : all) v.push_back(std::string(b));
        p.open(v);
      })
      .def("open_local", &PeerComm::open_local)
      .def("all_reduce", [](PeerComm& p, uintptr_t data, size_t n, DType t, uintptr_t st, RedOp op) {
        p.all_reduce(P<void>(data), n, t, S(st), op);
      }, py::arg("data"), py::arg("count"), py::arg("dtype"), py::arg("stream"), py::arg("op") = RedOp::kSum)
      .def("error", &PeerComm::error)
      .def("reset_error", &PeerComm::reset_error)
      .def("set_blocks", &PeerComm::set_blocks)
      .def("set_fence", &PeerComm::set_fence)
      .def("set_withhold", &PeerComm::set_withhold)
      .def("reset_state", &PeerComm::reset_state, py::call_guard<py::gil_scoped_release>())
      .def("set_timeout_ms", &PeerComm::set_timeout_ms)
      .def("set_oneshot_bytes", &PeerComm::set_oneshot_bytes)
      .def_property_readonly("oneshot_bytes", &PeerComm::oneshot_bytes)
      .def_property_readonly("blocks", &PeerComm::blocks)
      .def_property_readonly("fence", &PeerComm::fence)
      .def_property_readonly("rank", &PeerComm::rank)
      .def_property_readonly("world_size", &PeerComm::world_size)
      .def_property_readonly("mem_kind", &PeerComm::mem_kind)
      .def_property_readonly("cap_bytes", &PeerComm::cap_bytes)
      .def_static("partition", [](long long count, int ws, int blocks, int vec) {
        auto q = PeerPartition::make(count, ws, blocks, vec);
        return std::make_pair(q.chunk, q.slice);
      });

  m.def("set_dry_collectives", &reducer_set_dry,
        "every gradient Reducer skips its collectives (fences kept): the bench's compute-only pass");
  m.def("dry_collectives", &reducer_dry);
  py::class_<Reducer>(m, "Reducer")
      .def(py::init([](Comm* comm, uintptr_t flat, DType t, const std::vector<std::pair<size_t, size_t>>& buckets,
                       const std::vector<int>& param_bucket, RedOp op, bool timing) {
             std::vector<Reducer::BucketSpec> b;
             for (auto& x : buckets) b.push_back({x.first, x.second});
             return new Reducer(comm, flat, t, b, param_bucket, op, timing);
           }),
           py::arg("comm").none(true), py::arg("flat_grad"), py::arg("dtype"), py::arg("buckets"),
           py::arg("param_bucket"), py::arg("op") = RedOp::kSum, py::arg("timing") = false,
           py::keep_alive<1, 2>())
      .def("prepare", &Reducer::prepare)
      .def("abort", &Reducer::abort)
      .def("mark_ready", [](Reducer& r, int p, uintptr_t st) { r.mark_ready(p, S(st)); })
      .def("mark_bucket_ready", [](Reducer& r, int b, uintptr_t st) { r.mark_bucket_ready(b, S(st)); })
      .def("finalize", [](Reducer& r, uintptr_t st) { r.finalize(S(st)); })
      .def("comm_stream", [](Reducer& r) { return reinterpret_cast<uintptr_t>(r.comm_stream()); })
      .def("last_comm_ms", &Reducer::last_comm_ms)
      .def("set_timing", &Reducer::set_timing)
      .def("set_padding", &Reducer::set_padding)
      .def("padded_count", &Reducer::padded_count)
      .def("set_comm", &Reducer::set_comm, py::keep_alive<1, 2>())
      .def_property_readonly("timing", &Reducer::timing)
      .def_property_readonly("num_buckets", &Reducer::num_buckets)
      .def_property_readonly("launched", &Reducer::launched)
      .def("set_overlap", &Reducer::set_overlap)
      .def("set_peer", &Reducer::set_peer, py::arg("peer").none(true), py::keep_alive<1, 2>())
      .def("set_force_collectives", &Reducer::set_force_collectives)
      .def("set_comm_dtype", &Reducer::set_comm_dtype, py::arg("dtype"), py::arg("shadow") = 0)
      .def_property_readonly("comm_dtype", &Reducer::comm_dtype)
      .def_property_readonly("active", &Reducer::active);

  // ---------------------------------------------------------------- fused Keras-CNN engine
  m.def("keras_workspace_bytes", &KerasEngine::workspace_bytes);
  m.attr("KERAS_NUM_PARAMS") = KerasLayout::total;
  py::class_<KerasEngine>(m, "KerasEngine")
      .def(py::init([](int B, uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v, uintptr_t st, uintptr_t ws,
                       size_t wsb, Comm* comm, uint64_t seed, uintptr_t lr, uintptr_t metrics, float b1, float b2,
                       float eps, float wd, bool eps_hat) {
             return new KerasEngine(B, p, g, mm, v, st, ws, wsb, comm, seed, lr, metrics, b1, b2, eps, wd, eps_hat);
           }),
           py::arg("batch"), py::arg("params"), py::arg("grads"), py::arg("m"), py::arg("v"), py::arg("adam_state"),
           py::arg("workspace"), py::arg("workspace_bytes"), py::arg("comm").none(true), py::arg("seed"),
           py::arg("lr_dev"), py::arg("metrics_dev"), py::arg("b1"), py::arg("b2"), py::arg("eps"),
           py::arg("weight_decay"), py::arg("eps_hat"), py::keep_alive<1, 10>())
      .def("step", &KerasEngine::step)
      .def("capture", &KerasEngine::capture, py::arg("mode") = 1, py::arg("steps_per_graph") = 1)
      .def("replay", &KerasEngine::replay)
      .def("uncapture", &KerasEngine::uncapture)
      .def("warm_graphs", &KerasEngine::warm_graphs)
      .def("repack", &KerasEngine::repack)
      .def("sync", &KerasEngine::sync, py::call_guard<py::gil_scoped_release>())
      .def("set_peer", &KerasEngine::set_peer, py::arg("peer").none(true), py::keep_alive<1, 2>())
      .def("set_comm", &KerasEngine::set_comm, py::arg("comm").none(true), py::keep_alive<1, 2>())
      .def("set_force_collectives", &KerasEngine::set_force_collectives)
      .def("set_merged", &KerasEngine::set_merged)
      .def("set_overlap", &KerasEngine::set_overlap)
      .def("set_bucket_padding", &KerasEngine::set_bucket_padding)
      .def("set_external_batch", &KerasEngine::set_external_batch)
      .def("set_coscheduled", &KerasEngine::set_coscheduled)
      .def_property_readonly("coscheduled", &KerasEngine::coscheduled)
      .def_property_readonly("graph_mode", &KerasEngine::graph_mode)
      .def_property_readonly("merged", &KerasEngine::merged)
      .def_property_readonly("overlap", &KerasEngine::overlap)
      .def_property_readonly("world_size", &KerasEngine::world_size)
      .def_property_readonly("reducer_active", &KerasEngine::reducer_active)
      .def_property_readonly("peer_active", &KerasEngine::peer_active)
      .def_property_readonly("captured", &KerasEngine::captured)
      .def_property_readonly("stream", &KerasEngine::stream)
      .def_property_readonly("x_ptr", &KerasEngine::x_ptr)
      .def_property_readonly("y_ptr", &KerasEngine::y_ptr)
      .def_property_readonly("counter_ptr", &KerasEngine::counter_ptr);

  // ---------------------------------------------------------------- fused Chainer-MLP engine
  m.def("mlp_workspace_bytes", &MlpEngine::workspace_bytes);
  m.attr("MLP_NUM_PARAMS") = MlpLayout::total;
  m.attr("MLP_MAX_BATCH") = kMlpMaxBatch;
  py::class_<MlpEngine>(m, "MlpEngine")
      .def(py::init([](int B, uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v, uintptr_t st, uintptr_t ws,
                       size_t wsb, Comm* comm, uint64_t seed, uintptr_t lr, uintptr_t metrics, float b1, float b2,
                       float eps, float wd, bool eps_hat) {
             return new MlpEngine(B, p, g, mm, v, st, ws, wsb, comm, seed, lr, metrics, b1, b2, eps, wd, eps_hat);
           }),
           py::arg("batch"), py::arg("params"), py::arg("grads"), py::arg("m"), py::arg("v"), py::arg("adam_state"),
           py::arg("workspace"), py::arg("workspace_bytes"), py::arg("comm").none(true), py::arg("seed"),
           py::arg("lr_dev"), py::arg("metrics_dev"), py::arg("b1"), py::arg("b2"), py::arg("eps"),
           py::arg("weight_decay"), py::arg("eps_hat"), py::keep_alive<1, 10>())
      .def("step", &MlpEngine::step)
      .def("capture", &MlpEngine::capture, py::arg("mode") = 1, py::arg("steps_per_graph") = 1)
      .def("replay", &MlpEngine::replay)
      .def("uncapture", &MlpEngine::uncapture)
      .def("warm_graphs", &MlpEngine::warm_graphs)
      .def("sync", &MlpEngine::sync, py::call_guard<py::gil_scoped_release>())
      .def("set_peer", &MlpEngine::set_peer, py::arg("peer").none(true), py::keep_alive<1, 2>())
      .def("set_comm", &MlpEngine::set_comm, py::arg("comm").none(true), py::keep_alive<1, 2>())
      .def("set_force_collectives", &MlpEngine::set_force_collectives)
      .def("set_merged", &MlpEngine::set_merged)
      .def("set_overlap", &MlpEngine::set_overlap)
      .def("set_bucket_padding", &MlpEngine::set_bucket_padding)
      .def("set_external_batch", &MlpEngine::set_external_batch)
      .def_property_readonly("graph_mode", &MlpEngine::graph_mode)
      .def_property_readonly("merged", &MlpEngine::merged)
      .def_property_readonly("overlap", &MlpEngine::overlap)
      .def_property_readonly("world_size", &MlpEngine::world_size)
      .def_property_readonly("reducer_active", &MlpEngine::reducer_active)
      .def_property_readonly("peer_active", &MlpEngine::peer_active)
      .def_property_readonly("captured", &MlpEngine::captured)
      .def_property_readonly("stream", &MlpEngine::stream)
      .def_property_readonly("x_ptr", &MlpEngine::x_ptr)
      .def_property_readonly("y_ptr", &MlpEngine::y_ptr)
      .def_property_readonly("counter_ptr", &MlpEngine::counter_ptr);

  // ---------------------------------------------------------------- fused MNIST engine
  m.def("mnist_workspace_bytes", &MnistLayout::workspace_bytes);
  m.attr("MNIST_NUM_PARAMS") = MnistLayout::total;
  py::class_<MnistEngine>(m, "MnistEngine")
      .def(py::init([](int B, uintptr_t p, uintptr_t g, uintptr_t mom, uintptr_t ws, size_t wsb, Comm* comm,
                       uint64_t seed, float momentum, float wd, uintptr_t lr, uintptr_t metrics, int variant) {
             return new MnistEngine(B, p, g, mom, ws, wsb, comm, seed, momentum, wd, lr, metrics, variant);
           }),
           py::arg("batch"), py::arg("params"), py::arg("grads"), py::arg("mom"), py::arg("workspace"),
           py::arg("workspace_bytes"), py::arg("comm").none(true), py::arg("seed"), py::arg("momentum"),
           py::arg("weight_decay"), py::arg("lr_dev"), py::arg("metrics_dev"), py::arg("variant") = 1,
           py::keep_alive<1, 8>())
      .def("step", &MnistEngine::step)
      .def("capture", &MnistEngine::capture, py::arg("mode") = -1, py::arg("steps_per_graph") = 1)
      .def("set_force_collectives", &MnistEngine::set_force_collectives)
      .def_property_readonly("graph_mode", &MnistEngine::graph_mode)
      .def("set_overlap", &MnistEngine::set_overlap)
      .def("set_merged", &MnistEngine::set_merged)
      .def_property_readonly("merged", &MnistEngine::merged)
      .def("set_coscheduled", &MnistEngine::set_coscheduled)
      .def_property_readonly("coscheduled", &MnistEngine::coscheduled)
      .def("set_peer", &MnistEngine::set_peer, py::arg("peer").none(true), py::keep_alive<1, 2>())
      .def("set_comm", &MnistEngine::set_comm, py::arg("comm").none(true), py::keep_alive<1, 2>())
      .def("set_bucket_padding", &MnistEngine::set_bucket_padding)
      .def_property_readonly("peer_active", &MnistEngine::peer_active)
      .def_property_readonly("overlap", &MnistEngine::overlap)
      .def_property_readonly("reducer_active", &MnistEngine::reducer_active)
      .def("uncapture", &MnistEngine::uncapture)
      .def("replay", &MnistEngine::replay)
      .def("warm_graphs", &MnistEngine::warm_graphs)
      .def("set_small_first", &MnistEngine::set_small_first)
      .def("forward_only", &MnistEngine::forward_only)
      .def("repack", &MnistEngine::repack)
      .def("sync", &MnistEngine::sync, py::call_guard<py::gil_scoped_release>())
      .def("set_external_batch", &MnistEngine::set_external_batch)
      .def("set_trace", &MnistEngine::set_trace)
      .def("last_comm_ms", &MnistEngine::last_comm_ms)
      .def_property_readonly("stream", &MnistEngine::stream)
      .def_property_readonly("x_ptr", &MnistEngine::x_ptr)
      .def_property_readonly("y_ptr", &MnistEngine::y_ptr)
      .def_property_readonly("counter_ptr", &MnistEngine::counter_ptr)
      .def_property_readonly("captured", &MnistEngine::captured);
}
