#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ffk {

// Strided [B][H][S][D] views (element strides; D is contiguous). All pointers bf16.
struct AttnArgs {
  const uint16_t* q = nullptr; int64_t q_sb = 0, q_sh = 0, q_ss = 0;
  const uint16_t* k = nullptr; int64_t k_sb = 0, k_sh = 0, k_ss = 0;
  const uint16_t* v = nullptr; int64_t v_sb = 0, v_sh = 0, v_ss = 0;
  uint16_t* o = nullptr; int64_t o_sb = 0, o_sh = 0, o_ss = 0;
  float* lse = nullptr;  // [B*H][Sq]
  // backward
  const uint16_t* dout = nullptr; int64_t do_sb = 0, do_sh = 0, do_ss = 0;
  uint16_t* dq = nullptr; int64_t dq_sb = 0, dq_sh = 0, dq_ss = 0;
  uint16_t* dk = nullptr; int64_t dk_sb = 0, dk_sh = 0, dk_ss = 0;
  uint16_t* dv = nullptr; int64_t dv_sb = 0, dv_sh = 0, dv_ss = 0;
  float* dq_acc = nullptr;  // [ceil(Sk/128)][B*H][Sq][D] partials
  float* delta = nullptr;   // [B*H][Sq]
  float* lse2 = nullptr;    // [B*H][Sq] lse * log2(e) (attn_bwd_pre_kernel)
  // fused bias gradient of the [B,S,3,H,D] QKV projection: dbias [3][H][D] += column sums of dq /
  // dk / dv (attn_bwd1b_kernel partials in dbp, folded by attn_bias_fold_kernel); attn_bwd returns
  // whether it did, else the caller sums the bias gradient itself
  float* dbp = nullptr;
  float* dbias = nullptr;
  int B = 0, H = 0, Sq = 0, Sk = 0, D = 64;
  float scale = 1.f;
  int causal = 0;
  float rescale_thr = 8.f;  // forward: deferred-max threshold, log2 units (attn_set_rescale_thr)
  int stagger = 0;  // backward (attn_bwd1b_kernel): waves 4-7 run each dQ chunk after the softmax
};

void attn_fwd(AttnArgs a, hipStream_t st);
bool attn_bwd(AttnArgs a, hipStream_t st);
int64_t attn_bwd_workspace_floats(int B, int H, int Sq, int Sk, int D);
int64_t attn_bwd_slab_floats(int B, int H, int Sq, int Sk, int D);  // offset of delta in the workspace
int attn_bwd_variant();
void attn_set_bwd_variant(int v);
int attn_fwd_variant();
void attn_set_fwd_variant(int v);
float attn_rescale_thr();
int attn_stagger();
void attn_set_stagger(int v);
void attn_set_rescale_thr(float t);

}  // namespace ffk
