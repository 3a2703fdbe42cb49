// pybind11 module `_nidt_hip`: host entry points of the gfx950 kernels in csrc/kernels/*.hip.
// Every function takes raw device pointers (uintptr_t), sizes and a hipStream_t (as uintptr_t); shape and dtype
// validation happens in the Python wrappers (neuroimagedisttraining_amd/ops) before any launch.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <cstdint>
#include <vector>

namespace nidt {
// optim.hip
int64_t clip_sgd_mask_workspace(int64_t C, int64_t P);
void clip_sgd_mask(uintptr_t w, uintptr_t g, uintptr_t buf, uintptr_t mask, uintptr_t part, uintptr_t coef_out,
                   uintptr_t wbf, int64_t C, int64_t P, int64_t stride, float lr, float wd, float mom, int first,
                   float max_norm, uintptr_t lr_dev, int keep_grad, uintptr_t stream);
int64_t rows_nnz_blocks(int64_t P);
void rows_nnz(uintptr_t rows, int64_t R, int64_t P, int64_t stride, uintptr_t part, uintptr_t stream);
void weighted_rows_sum(uintptr_t rows, uintptr_t wts, int64_t C, int64_t P, int64_t stride, float beta, uintptr_t out,
                       uintptr_t stream);
void broadcast_row(uintptr_t src, int64_t P, int64_t stride, int64_t C, uintptr_t dst, uintptr_t stream);
void local_opt(uintptr_t w, uintptr_t g, uintptr_t buf, int64_t ld, uintptr_t mbits, int64_t mstride, int mask_mode,
               uintptr_t ref, int64_t ref_ld, float mu, uintptr_t pref, int64_t pref_ld, float lamda, uintptr_t part,
               int64_t C, int64_t P, float lr, float wd, float mom, float max_norm, uintptr_t lr_dev, int keep_grad,
               uintptr_t stream);
void local_opt_pack(uintptr_t w, uintptr_t g, uintptr_t buf, int64_t ld, uintptr_t mbits, int64_t mstride,
                    int mask_mode, uintptr_t ref, int64_t ref_ld, float mu, uintptr_t pref, int64_t pref_ld,
                    float lamda, uintptr_t part, int64_t C, int64_t P, float lr, float wd, float mom, float max_norm,
                    uintptr_t lr_dev, int keep_grad, uintptr_t desc, int nd, int nconv, uintptr_t rest, int nrest,
                    int lds, uintptr_t out, uintptr_t stream);
void local_opt_pack_wt(uintptr_t w, uintptr_t g, uintptr_t buf, int64_t ld, uintptr_t mbits, int64_t mstride,
                       int mask_mode, uintptr_t ref, int64_t ref_ld, float mu, uintptr_t pref, int64_t pref_ld,
                       float lamda, uintptr_t part, int64_t C, int64_t P, float lr, float wd, float mom, float max_norm,
                       uintptr_t lr_dev, int keep_grad, uintptr_t desc, int nd, int nconv, uintptr_t rest, int nrest,
                       int lds, uintptr_t out, uintptr_t stream);
int wt_tiles(int cout, int cin_p);
int wt_tile_lds(int kt);
// conv3d.hip
void conv3d_fwd(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t xs, uintptr_t xt, uintptr_t y, uintptr_t stats,
                int G, int B, int D, int H, int W, int Cin, int Cout, int pad, uintptr_t stream);
void conv3d_fwd_splitk(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, uintptr_t stats, uintptr_t part,
                       int ksplit, int G, int B, int D, int H, int W, int Cin, int Cout, int pad, uintptr_t stream);
int conv3d_fwd_ksplit(int Cin, int Cout, int G, int Mg);
void conv3d_fwd_bld(uintptr_t x, uintptr_t w, uintptr_t bias, int64_t bias_ld, uintptr_t y, uintptr_t stats, int G, int B,
                    int D, int H, int W, int Cin, int Cout, int pad, uintptr_t stream);
int conv3d_fwd_nblocks(int B, int D, int H, int W, int pad, int bp);
int conv3d_fwd_bp(int Cin, int Cout, int xf, int G, int Mg);
void conv3d_wgrad(uintptr_t x, uintptr_t xs, uintptr_t xt, uintptr_t dy, uintptr_t part, uintptr_t grad, int64_t ldg,
                  int64_t off, int G, int B, int D, int H, int W, int Cin, int Cout, int pad, int nsplit, float scale,
                  uintptr_t ptab, uintptr_t stream);
void conv3d_pos_table(uintptr_t tab, int B, int D, int H, int W, int pad, uintptr_t stream);
int conv3d_wgrad_nsplit(int G, int B, int D, int H, int W, int Cin, int Cout, int pad);
int conv3d_wgrad_tri_table_size(int B, int D, int H, int W, int pad);
int conv3d_wgrad_slab_ok(int B, int D, int H, int W, int Cin, int Cout, int pad);
int conv3d_wgrad_slab_pick(int G, int B, int D, int H, int W, int Cin, int Cout, int pad);
int conv3d_wgrad_slab_nsplit(int G, int B, int D, int H, int W, int Cin, int Cout, int pad);
int conv3d_wgrad_slab_table_size(int B, int D, int H, int W, int pad);
void conv3d_wgrad_slab_table(uintptr_t tab, int B, int D, int H, int W, int pad, uintptr_t stream);
void conv3d_wgrad_slab(uintptr_t x, uintptr_t dy, uintptr_t part, uintptr_t grad, int64_t ldg, int64_t off, int G,
                       int B, int D, int H, int W, int Cin, int Cout, int pad, int nsplit, float scale, uintptr_t stab,
                       uintptr_t stream);
int conv3d_fwd_tri_ok(int B, int D, int H, int W, int Cin, int Cout, int pad);
int conv3d_union_umax(int B, int D, int H, int W, int pad, int P);
int conv3d_fwd_tri_pick(int G, int B, int D, int H, int W, int Cin, int Cout, int pad);
int conv3d_fwd_tri_table_size(int B, int D, int H, int W, int pad);
int conv3d_fwd_slab_ok(int B, int D, int H, int W, int Cin, int Cout, int pad);
int conv2d_fwd_slab_ok(int B, int H, int W, int Cin, int Cout);
int conv3d_fwd_vol_ok(int B, int D, int H, int W, int Cin, int Cout, int pad);
int conv3d_fwd_vol_pick(int G, int B, int D, int H, int W, int Cin, int Cout, int pad);
void conv3d_fwd_vol(uintptr_t x, uintptr_t w, uintptr_t bias, int64_t bias_ld, uintptr_t y, uintptr_t stats, int G,
                    int B, int D, int H, int W, int Cin, int Cout, int pad, uintptr_t stream);
void unpack_bits_dev(uintptr_t bits, int64_t mstride, int64_t R, int64_t P, int f32, uintptr_t out, uintptr_t stream);
void masked_rows(uintptr_t src, uintptr_t bits, int64_t mstride, int64_t C, int64_t P, int64_t ld, uintptr_t dst,
                 uintptr_t stream);
void stream_fork(uintptr_t src, uintptr_t dst);
int conv2d_fwd_slab_bd_ok(int B, int H, int W, int Cin, int Cout);
int conv2d_fwd_slab_bd_pick(int G, int B, int H, int W, int Cin, int Cout);
int conv2d_fwd_slab_bd_table_size(int B, int H, int W, int Cin, int Cout);
void conv2d_fwd_slab_bd_table(uintptr_t tab, int B, int H, int W, int Cin, int Cout, uintptr_t stream);
void conv2d_fwd_slab_bd(uintptr_t x, uintptr_t w, uintptr_t y, int G, int B, int H, int W, int Cin, int Cout,
                        uintptr_t utab, uintptr_t stream);
int conv2d_fwd_slab_pick(int G, int B, int H, int W, int Cin, int Cout);
void conv2d_fwd_slab_stats(uintptr_t x, uintptr_t w, uintptr_t zb, uintptr_t y, uintptr_t stats, int G, int B, int H,
                           int W, int Cin, int Cout, uintptr_t utab, uintptr_t stream);
void gn_apply(uintptr_t t, uintptr_t res, uintptr_t part, int nb, int bp, uintptr_t theta, int64_t ldt, int64_t off_w,
              int64_t off_b, uintptr_t y, uintptr_t stats, int N, int B, int S, int C, int relu, uintptr_t stream);
void conv2d_fwd_slab(uintptr_t x, uintptr_t w, uintptr_t y, int G, int B, int H, int W, int Cin, int Cout,
                     uintptr_t utab, uintptr_t stream);
int conv3d_slab_umax(int B, int D, int H, int W, int pad);
int conv3d_fwd_slab_pick(int G, int B, int D, int H, int W, int Cin, int Cout, int pad);
int conv3d_fwd_slab_table_size(int B, int D, int H, int W, int pad);
void conv3d_fwd_slab_table(uintptr_t tab, int B, int D, int H, int W, int pad, uintptr_t stream);
void conv3d_fwd_slab(uintptr_t x, uintptr_t w, uintptr_t bias, int64_t bias_ld, uintptr_t y, uintptr_t stats, int G,
                     int B, int D, int H, int W, int Cin, int Cout, int pad, uintptr_t utab, uintptr_t stream);
void conv3d_fwd_tri_table(uintptr_t tab, int B, int D, int H, int W, int pad, uintptr_t stream);
void conv3d_fwd_tri(uintptr_t x, uintptr_t w, uintptr_t bias, int64_t bias_ld, uintptr_t y, uintptr_t stats, int G,
                    int B, int D, int H, int W, int Cin, int Cout, int pad, uintptr_t utab, uintptr_t stream);
int conv3d_wgrad_tri_nsplit(int G, int B, int D, int H, int W, int Cin, int Cout, int pad);
void conv3d_wgrad_tri_table(uintptr_t tab, int B, int D, int H, int W, int pad, uintptr_t stream);
int conv3d_wgrad_tri_ok(int B, int D, int H, int W, int Cin, int Cout, int pad);
int conv3d_wgrad_tri_pick(int G, int B, int D, int H, int W, int Cin, int Cout, int pad);
void conv3d_wgrad_tri(uintptr_t x, uintptr_t dy, uintptr_t part, uintptr_t grad, int64_t ldg, int64_t off, int G, int B,
                      int D, int H, int W, int Cin, int Cout, int pad, int nsplit, float scale, uintptr_t stab,
                      uintptr_t stream);
void pack_conv_w(uintptr_t theta, int64_t ldt, int64_t off, int G, int Cout, int Cin, float scale, uintptr_t wp,
                 uintptr_t wt, uintptr_t stream);
void bn_relu_apply(uintptr_t y, uintptr_t sc, uintptr_t sh, uintptr_t h, int64_t npos, int C, int S, uintptr_t stream);
void conv_fwd_g(uintptr_t x, uintptr_t w, uintptr_t y, int G, int B, int D, int H, int W, int Cin, int Cout, int kt,
                int st, int pad, int padd, uintptr_t stream);
int conv_fwd_g_ksplit(int G, int B, int D, int H, int W, int Cin, int Cout, int kt, int st, int pad, int padd);
void conv_fwd_gk(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t part, int ksplit, int G, int B, int D, int H, int W,
                 int Cin, int Cout, int kt, int st, int pad, int padd, uintptr_t stream);
void conv_pos_table_g(uintptr_t tab, int B, int D, int H, int W, int kt, int st, int pad, int padd, uintptr_t stream);
void conv_wgrad_g(uintptr_t x, uintptr_t dy, uintptr_t part, uintptr_t grad, int64_t ldg, int64_t off, int G, int B,
                  int D, int H, int W, int Cin, int Cout, int kt, int st, int pad, int padd, int nsplit, float scale,
                  uintptr_t ptab, uintptr_t stream);
int conv_wgrad_nsplit_g(int G, int B, int D, int H, int W, int Cin, int Cout, int kt, int st, int pad, int padd);
void pack_conv_wk(uintptr_t theta, int64_t ldt, int64_t off, int G, int Cout, int Cin, int kt, int cin_src,
                  float scale, uintptr_t wp, uintptr_t wt, uintptr_t stream);
// gn.hip
void gn_fwd(uintptr_t t, uintptr_t res, uintptr_t theta, int64_t ldt, int64_t off_w, int64_t off_b, uintptr_t y,
            uintptr_t stats, int N, int B, int S, int C, int relu, uintptr_t stream);
void gn_bwd_rm(uintptr_t dy, int dy_bf16, uintptr_t t, uintptr_t stats, uintptr_t theta, int64_t ldt, int64_t off_w,
               int64_t off_b, uintptr_t dt, uintptr_t part, int N, int B, int S, int C, uintptr_t stream);
int gn_rm_ok(int S, int C);
void gn_bwd(uintptr_t dy, int dy_bf16, uintptr_t mask, uintptr_t t, uintptr_t stats, uintptr_t theta, int64_t ldt,
            int64_t off_w, uintptr_t dt, uintptr_t part, int N, int B, int S, int C, uintptr_t stream);
void gn_param_grads(uintptr_t part, int G, int B, int C, uintptr_t grads, int64_t ldg, int64_t off_w, int64_t off_b,
                    uintptr_t stream);
void res_grad(uintptr_t out, uintptr_t dx1, uintptr_t dx2, uintptr_t da, uintptr_t mask, int64_t n, int flags,
              uintptr_t stream);
void res_grad_s2(uintptr_t out, uintptr_t dx1, uintptr_t dx2s, int N, int D, int H, int W, int C, int out_bf16,
                 uintptr_t stream);
void res_grad_om(uintptr_t out, uintptr_t dx1, uintptr_t dx2, uintptr_t da, uintptr_t mask, uintptr_t omask, int64_t n,
                 int flags, uintptr_t stream);
void res_grad_s2_om(uintptr_t out, uintptr_t dx1, uintptr_t dx2s, uintptr_t omask, int N, int D, int H, int W, int C,
                    int out_bf16, uintptr_t stream);
// img.hip
void img_input(uintptr_t src, uintptr_t idx, uintptr_t out, int N, int H, int W, int CP, float m0, float m1, float m2,
               float s0, float s1, float s2, int aug, int pad, uintptr_t seed_dev, int64_t seed_base, uintptr_t cids,
               int B, uintptr_t stream);
void img_input_fold(uintptr_t src, uintptr_t idx, uintptr_t out, int N, int H, int W, int CP, float m0, float m1,
                    float m2, float s0, float s1, float s2, int aug, int pad, uintptr_t seed_dev, int64_t seed_base,
                    uintptr_t cids, int B, uintptr_t stream);
// pack.hip
void pack_convs(uintptr_t desc, int nd, int nplain, int nplain1, int ntrans, int lds, uintptr_t theta, int64_t ldt,
                int G, uintptr_t out, uintptr_t stream);
int pack1_rows_host(int cin_p);
int pack_plain_chunks(int cin_p, int kt);
int pack_plain_lds(int cin_p, int kt);
int pack_desc_bytes();
// conv3d.hip (sub-pixel stride-2 data gradient)
void conv_dgrad_s2_g(uintptr_t dy, uintptr_t w, uintptr_t dx, int G, int B, int D, int H, int W, int Cin, int Cout,
                     int kt, int Dx, int Hx, int Wx, uintptr_t stream);
std::vector<int> conv_tap_slots(int kt, int stride);
// mpc.hip
void modp_matmul(uintptr_t A, uintptr_t B, uintptr_t C, int M, int K, int64_t N, int64_t p, uintptr_t stream);
// bnr.hip
int bnr_workspace(int G, int64_t M, int C);
void bnr_stats(uintptr_t t, int G, int64_t M, int C, float eps, float mom, uintptr_t ws, uintptr_t stats,
               uintptr_t bufs, int64_t ldb, int64_t off_rm, int64_t off_rv, int64_t off_nbt, uintptr_t stream);
void bnr_eval_stats(int G, int C, float eps, uintptr_t bufs, int64_t ldb, int64_t off_rm, int64_t off_rv,
                    uintptr_t stats, uintptr_t stream);
void bnr_apply(uintptr_t t, uintptr_t res, uintptr_t stats, uintptr_t theta, int64_t ldt, int64_t off_w, int64_t off_b,
               uintptr_t y, int G, int64_t M, int C, int relu, uintptr_t stream);
void bnr_bwd(uintptr_t t, uintptr_t dy, int dy_bf16, uintptr_t mask, uintptr_t stats, uintptr_t theta, int64_t ldt,
             int64_t off_w, int64_t off_b, uintptr_t grads, int64_t ldg, uintptr_t ws, uintptr_t coef, uintptr_t dt,
             int G, int64_t M, int C, int eval_mode, uintptr_t stream);
void bnr_bwd_tm(uintptr_t t, uintptr_t dy, int dy_bf16, uintptr_t mask, uintptr_t stats, uintptr_t theta, int64_t ldt,
                int64_t off_w, int64_t off_b, uintptr_t grads, int64_t ldg, uintptr_t ws, uintptr_t coef, uintptr_t dt,
                int G, int64_t M, int C, int eval_mode, int tmask, uintptr_t stream);
void bnr_res_partial(uintptr_t out, uintptr_t dx1, uintptr_t dx2, uintptr_t da, uintptr_t mask, uintptr_t omask,
                     uintptr_t t3, uintptr_t s3, uintptr_t ws3, uintptr_t td, uintptr_t sd, uintptr_t wsd, int G,
                     int64_t M, int C, uintptr_t stream);
void bnr_bwd_part(uintptr_t t, uintptr_t dy, uintptr_t stats, uintptr_t theta, int64_t ldt, int64_t off_w,
                  int64_t off_b, uintptr_t grads, int64_t ldg, uintptr_t ws, uintptr_t coef, uintptr_t dt, int G,
                  int64_t M, int C, uintptr_t stream);
// bn.hip
void bn_finalize(uintptr_t stats, int nPB, int BP, int Mg, int G, int C, uintptr_t theta, int64_t ldt, int64_t off_g,
                 int64_t off_b, uintptr_t bufs, int64_t ldb, int64_t off_rm, int64_t off_rv, int64_t off_nbt,
                 float momentum, float eps, uintptr_t scale, uintptr_t shift, uintptr_t mean, uintptr_t invstd,
                 int update_running, uintptr_t stream);
void bn_eval(int G, int C, uintptr_t theta, int64_t ldt, int64_t off_g, int64_t off_b, uintptr_t bufs, int64_t ldb,
             int64_t off_rm, int64_t off_rv, float eps, uintptr_t scale, uintptr_t shift, uintptr_t mean,
             uintptr_t invstd, uintptr_t stream);
void bn_relu_pool(uintptr_t y, uintptr_t scale, uintptr_t shift, uintptr_t out, uintptr_t amax, int NB, int B, int D,
                  int H, int W, int C, uintptr_t stream);
void bn_bwd(int pool, uintptr_t y, uintptr_t dsrc, uintptr_t pout, uintptr_t amax, uintptr_t scale, uintptr_t shift,
            uintptr_t mean, uintptr_t invstd, int NB, int B, int D, int H, int W, int C, uintptr_t part, int nchunk,
            uintptr_t theta, int64_t ldt, int64_t off_g, uintptr_t grad, int64_t ldg, int64_t goff_g, int64_t goff_b,
            int64_t goff_convb, uintptr_t coef, uintptr_t dy, int eval_mode, uintptr_t stream);
// conv1.hip
void polyphase(uintptr_t src, uintptr_t dst, int64_t N, uintptr_t stream);
void conv1_sample_moments(uintptr_t x8, int64_t N, uintptr_t mom, uintptr_t stream);
void pack_conv1_w(uintptr_t theta, int64_t ldt, int64_t off, int64_t off_sign, int G, float scale, uintptr_t w8,
                  uintptr_t w125,
                  uintptr_t stream);
void conv1_bnstats(uintptr_t mom, uintptr_t idx, int B, int G, uintptr_t Mb, uintptr_t w125, uintptr_t theta,
                   int64_t ldt, int64_t off_bias, int64_t off_g, int64_t off_b, uintptr_t bufs, int64_t ldb,
                   int64_t off_rm, int64_t off_rv, int64_t off_nbt, float momentum, float eps, int update_running,
                   uintptr_t scale, uintptr_t shift, uintptr_t mean, uintptr_t invstd, uintptr_t mu, uintptr_t covw,
                   uintptr_t stream);
void conv1_fwd_pool(uintptr_t x8, uintptr_t idx, uintptr_t w8, uintptr_t scale, uintptr_t shift, int NB, int B,
                    uintptr_t out, uintptr_t amax, uintptr_t stream);
int conv1_wgrad_nq(int NB);
int conv1_wgrad_mx_npb(int NB);
void conv1_wgrad_mode(int mode);
void conv1_fwd_mode(int mode);
int gemm1x1_ok(int K, int N);
int wgrad1x1_ok(int N, int K);
int wgrad1x1_chunks(int G, int64_t Mg, int N, int K);
void wgrad1x1_g(uintptr_t x, uintptr_t dy, uintptr_t part, uintptr_t grad, int64_t ldg, int64_t off, int G, int64_t Mg,
                int N, int K, int nMB, float scale, uintptr_t stream);
void conv2d_any_fwd(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int G, int B, int H, int W, int cin, int cs,
                    int cout, int k, int pad, uintptr_t stream);
int conv2d_any_wgrad_chunks(int B, int Ho, int Wo);
void conv2d_any_wgrad(uintptr_t x, uintptr_t dy, uintptr_t part, int G, int B, int H, int W, int cin, int cs, int cout,
                      int k, int pad, uintptr_t stream);
int gemm1x1_chunks(int G, int64_t Mg, int K, int N);
void gemm1x1_g(uintptr_t x, uintptr_t w, uintptr_t y, int G, int64_t Mg, int K, int N, uintptr_t part,
               uintptr_t stream);
void bnr_finalize_part(uintptr_t part, int nchunk, int G, int64_t M, int C, float eps, float mom, uintptr_t stats,
                       uintptr_t bufs, int64_t ldb, int64_t off_rm, int64_t off_rv, int64_t off_nbt, uintptr_t stream);
int conv1_kslots();
void conv1_wgrad(uintptr_t x8, uintptr_t idx, uintptr_t dp, uintptr_t pout, uintptr_t amax, int NB, int B,
                 uintptr_t part, uintptr_t w125, uintptr_t mu, uintptr_t covw, uintptr_t invstd, uintptr_t theta,
                 int64_t ldt, int64_t off_g, uintptr_t grad, int64_t ldg, int64_t goff_w, int64_t goff_bias,
                 int64_t goff_g, int64_t goff_b, float wscale, uintptr_t emean, uintptr_t stream);
// head.hip
void cls_head_train(uintptr_t a, uintptr_t theta, int64_t ldt, int64_t off_w, int64_t off_b, uintptr_t y, int G, int B,
                    int HW, int C, int K, uintptr_t pooled, uintptr_t dlog, uintptr_t lossn, uintptr_t losses,
                    uintptr_t grad, int64_t ldg, uintptr_t da, uintptr_t stream);
void head(uintptr_t p5, uintptr_t theta, int64_t ldt, int64_t off_w1, int64_t off_b1, int64_t off_w2, int64_t off_b2,
          uintptr_t y, uintptr_t logits, uintptr_t loss, uintptr_t grad, int64_t ldg, uintptr_t dp5, int G, int B,
          int train, float keep, uint64_t seed, uintptr_t cids, uintptr_t seed_dev, uintptr_t stream);
// select.hip
void saliency_acc(uintptr_t theta, uintptr_t grad, int64_t ld, int64_t P, int G, float alpha, uintptr_t score,
                  int64_t lds, uintptr_t stream);
void radix_select_kth(uintptr_t v, int64_t n, int64_t k, uintptr_t state, uintptr_t hist, uintptr_t stream);
void threshold_mask(uintptr_t v, int64_t n, uintptr_t state, uintptr_t mask, uintptr_t stream);
void mask_stats(uintptr_t a, uintptr_t b, int64_t n, uintptr_t out, uintptr_t stream);
// sparse.hip
void seg_count(uintptr_t tiles, int ntiles, uintptr_t A, uintptr_t Bm, int64_t mstride, uintptr_t v, int64_t ldv,
               int mode, int S, uintptr_t out, uintptr_t stream);
void seg_select(uintptr_t tiles, uintptr_t tile_first, int ntiles, uintptr_t v, int64_t ldv, uintptr_t bits,
                int64_t mstride, uintptr_t cids, uint64_t seed, int R, int S, int mode, uintptr_t state,
                uintptr_t hist, uintptr_t ties, int query_only, uintptr_t stream);
void seg_prune(uintptr_t tiles, int ntiles, uintptr_t v, int64_t ldv, uintptr_t out, int64_t mstride, uintptr_t thr,
               uintptr_t prune, int S, uintptr_t stream);
void masked_rows_sum(uintptr_t rows, int64_t ld, uintptr_t bits, int64_t mstride, int R, int64_t n, uintptr_t sum,
                     uintptr_t cnt, uintptr_t stream);
void mix_rows(uintptr_t src, uintptr_t wts, uintptr_t rowptr, uintptr_t dst, int R, int64_t n, uintptr_t stream);
void masked_mean_rows(uintptr_t src, uintptr_t sbits, uintptr_t rp, uintptr_t dst, uintptr_t own, int R, int64_t n,
                      uintptr_t stream);
int pair_sqdist_nblk(int64_t n);
void pair_sqdist(uintptr_t pa, uintptr_t pb, int K, int64_t n, uintptr_t part, uintptr_t stream);
void stem_polyphase(uintptr_t src, uintptr_t idx, int N, int D, int H, int W, uintptr_t xp, uintptr_t xq,
                    uintptr_t stream);
void stem_fwd(uintptr_t xp, uintptr_t theta, int64_t ldt, int64_t off_w, int N, int B, int D, int H, int W, uintptr_t wk,
              uintptr_t y, uintptr_t stats, uintptr_t stream);
void stem_pool(uintptr_t y, uintptr_t scale, uintptr_t shift, int N, int B, int D, int H, int W, uintptr_t out,
               uintptr_t amax, uintptr_t stream);
void stem_bwd(uintptr_t dpool, uintptr_t amax, uintptr_t y, uintptr_t xq, uintptr_t scale, uintptr_t shift,
              uintptr_t mean, uintptr_t invstd, int N, int B, int D, int H, int W, uintptr_t theta, int64_t ldt,
              int64_t off_g, uintptr_t grad, int64_t ldg, int64_t goff_w, int64_t goff_g, int64_t goff_b, uintptr_t dz,
              uintptr_t part, uintptr_t coef, uintptr_t slab, uintptr_t stream);
std::vector<int64_t> stem_sizes(int N, int D, int H, int W);
}  // namespace nidt

PYBIND11_MODULE(_nidt_hip, m) {
  m.doc() = "gfx950 (MI355X) HIP kernels of neuroimagedisttraining_amd";
  m.attr("ARCH") = "gfx950";
#define DEF(name) m.def(#name, &nidt::name)
  DEF(clip_sgd_mask_workspace);
  DEF(clip_sgd_mask);
  DEF(weighted_rows_sum);
  DEF(rows_nnz_blocks);
  DEF(rows_nnz);
  DEF(broadcast_row);
  DEF(conv3d_fwd);
  DEF(conv3d_fwd_splitk);
  DEF(conv3d_fwd_ksplit);
  DEF(conv3d_fwd_bld);
  DEF(conv3d_fwd_nblocks);
  DEF(conv3d_fwd_bp);
  DEF(conv3d_wgrad);
  DEF(conv3d_wgrad_nsplit);
  DEF(conv3d_wgrad_tri_table_size);
  DEF(conv3d_fwd_tri_ok);
  DEF(conv3d_union_umax);
  DEF(conv3d_fwd_tri_pick);
  DEF(conv3d_fwd_tri_table_size);
  DEF(conv3d_fwd_tri_table);
  DEF(conv3d_fwd_tri);
  DEF(conv3d_fwd_slab_ok);
  DEF(conv3d_slab_umax);
  DEF(conv3d_fwd_slab_pick);
  DEF(conv3d_fwd_slab_table_size);
  DEF(conv3d_fwd_slab_table);
  DEF(conv3d_fwd_slab);
  DEF(conv2d_fwd_slab_ok);
  DEF(conv3d_fwd_vol_ok);
  DEF(conv3d_fwd_vol_pick);
  DEF(conv3d_fwd_vol);
  DEF(unpack_bits_dev);
  DEF(masked_rows);
  DEF(stream_fork);
  DEF(conv2d_fwd_slab_bd_ok);
  DEF(conv2d_fwd_slab_bd_pick);
  DEF(conv2d_fwd_slab_bd_table_size);
  DEF(conv2d_fwd_slab_bd_table);
  DEF(conv2d_fwd_slab_bd);
  DEF(conv2d_fwd_slab_pick);
  DEF(conv2d_fwd_slab);
  DEF(conv2d_fwd_slab_stats);
  DEF(gn_apply);
  DEF(conv3d_wgrad_tri_nsplit);
  DEF(conv3d_wgrad_tri_table);
  DEF(conv3d_wgrad_tri_ok);
  DEF(conv3d_wgrad_tri_pick);
  DEF(conv3d_wgrad_tri);
  DEF(conv3d_wgrad_slab_ok);
  DEF(conv3d_wgrad_slab_pick);
  DEF(conv3d_wgrad_slab_nsplit);
  DEF(conv3d_wgrad_slab_table_size);
  DEF(conv3d_wgrad_slab_table);
  DEF(conv3d_wgrad_slab);
  DEF(conv3d_pos_table);
  DEF(pack_conv_w);
  DEF(bn_relu_apply);
  DEF(conv_fwd_g);
  DEF(conv_fwd_g_ksplit);
  DEF(conv_fwd_gk);
  DEF(conv_pos_table_g);
  DEF(conv_wgrad_g);
  DEF(conv_wgrad_nsplit_g);
  DEF(pack_conv_wk);
  DEF(gn_fwd);
  DEF(gn_bwd);
  DEF(gn_bwd_rm);
  DEF(gn_rm_ok);
  DEF(gn_param_grads);
  DEF(res_grad_om);
  DEF(res_grad_s2_om);
  DEF(res_grad);
  DEF(res_grad_s2);
  DEF(img_input);
  DEF(img_input_fold);
  DEF(pack_convs);
  DEF(pack1_rows_host);
  DEF(pack_plain_chunks);
  DEF(pack_plain_lds);
  DEF(pack_desc_bytes);
  DEF(conv_dgrad_s2_g);
  DEF(conv_tap_slots);
  DEF(modp_matmul);
  DEF(bnr_workspace);
  DEF(bnr_stats);
  DEF(bnr_eval_stats);
  DEF(bnr_apply);
  DEF(bnr_res_partial);
  DEF(bnr_bwd_part);
  DEF(bnr_bwd_tm);
  DEF(bnr_bwd);
  DEF(bn_finalize);
  DEF(bn_eval);
  DEF(bn_relu_pool);
  DEF(bn_bwd);
  DEF(polyphase);
  DEF(conv1_sample_moments);
  DEF(pack_conv1_w);
  DEF(conv1_bnstats);
  DEF(conv1_fwd_pool);
  DEF(conv1_wgrad);
  DEF(conv1_wgrad_nq);
  DEF(conv1_wgrad_mx_npb);
  DEF(conv1_wgrad_mode);
  DEF(conv1_fwd_mode);
  DEF(gemm1x1_ok);
  DEF(wgrad1x1_ok);
  DEF(wgrad1x1_chunks);
  DEF(wgrad1x1_g);
  DEF(conv2d_any_fwd);
  DEF(conv2d_any_wgrad_chunks);
  DEF(conv2d_any_wgrad);
  DEF(gemm1x1_g);
  DEF(gemm1x1_chunks);
  DEF(bnr_finalize_part);
  DEF(conv1_kslots);
  DEF(head);
  DEF(cls_head_train);
  DEF(saliency_acc);
  DEF(radix_select_kth);
  DEF(threshold_mask);
  DEF(mask_stats);
  DEF(local_opt);
  DEF(local_opt_pack);
  DEF(local_opt_pack_wt);
  DEF(wt_tiles);
  DEF(wt_tile_lds);
  DEF(seg_count);
  DEF(seg_select);
  DEF(seg_prune);
  DEF(masked_rows_sum);
  DEF(mix_rows);
  DEF(masked_mean_rows);
  DEF(pair_sqdist_nblk);
  DEF(pair_sqdist);
  DEF(stem_polyphase);
  DEF(stem_fwd);
  DEF(stem_pool);
  DEF(stem_bwd);
  DEF(stem_sizes);
#undef DEF
}
