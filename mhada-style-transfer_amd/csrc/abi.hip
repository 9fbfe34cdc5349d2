// C-ABI plumbing shared by every entry point: thread-local error message, launch checks, the
// kernel-variant table (read once at the first launch, see Tuning in common.h).
#include "common.h"

#include <mutex>
#include <stdlib.h>
#include <string.h>

namespace mhada {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(const std::string& msg) {
  set_error(msg);
  return MHADA_ERR_ARG;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return MHADA_ERR_LAUNCH;
  }
  return MHADA_OK;
}

namespace {
struct Knob {
  const char* name;  // mhada_set_tuning name; env variable MHADA_<NAME upper-cased>
  int Tuning::*field;
};
const Knob kKnobs[] = {
    {"attn_fixed_shift", &Tuning::attn_fixed_shift}, {"attn_waves", &Tuning::attn_waves},
    {"attn_tk", &Tuning::attn_tk},                   {"attn_prio", &Tuning::attn_prio},
    {"vit_attn_vec", &Tuning::vit_attn_vec},         {"out3_mfma", &Tuning::out3_mfma},
    {"out3_tile", &Tuning::out3_tile},               {"gemm_pp", &Tuning::gemm_pp},
    {"gemm_persist", &Tuning::gemm_persist},         {"gemm_pp128", &Tuning::gemm_pp128},
    {"gemm_ldsepi", &Tuning::gemm_ldsepi},           {"gemm_n64", &Tuning::gemm_n64},
    {"conv_c64", &Tuning::conv_c64},                 {"conv_dir", &Tuning::conv_dir},                 {"gemm_rinit", &Tuning::gemm_rinit},
    {"tn_skinny_lds", &Tuning::tn_skinny_lds},       {"train_dkv_dma", &Tuning::train_dkv_dma},
    {"wino4", &Tuning::wino4},                       {"upsample_quad", &Tuning::upsample_quad},
    {"xknob", &Tuning::xknob},
};

Tuning g_tuning;
std::once_flag g_tuning_once;

void read_env_once() {
  std::call_once(g_tuning_once, [] {
    for (const Knob& k : kKnobs) {
      std::string env = "MHADA_";
      for (const char* c = k.name; *c; ++c) env += (char)(*c >= 'a' && *c <= 'z' ? *c - 32 : *c);
      if (const char* v = getenv(env.c_str())) g_tuning.*k.field = atoi(v);
    }
  });
}

bool valid(const char* name, int v) {
  if (!strcmp(name, "attn_waves")) return v == 0 || v == 4 || v == 8;
  if (!strcmp(name, "attn_tk")) return v == 64 || v == 128;
  if (!strcmp(name, "gemm_n64")) return v == 128 || v == 256;
  if (!strcmp(name, "xknob")) return v >= 0 && v < 16;
  return v == 0 || v == 1;
}
}  // namespace

const Tuning& tuning() {
  read_env_once();
  return g_tuning;
}

}  // namespace mhada

extern "C" int mhada_abi_version(void) { return 16; }  // 16: mhada_split3_kv / mhada_kv_proj_split3 / mhada_attn_split3 / mhada_attn_train_fwd_split3 (the fp32 softmax MHAda attention as SPLIT3 products on the bf16 MFMA); 15: mhada_gemm a_mode MHADA_A_SPLIT3 (fp32-accurate products on the bf16 MFMA), mhada_layernorm y_dtype MHADA_BF16X3; 14: mhada_cosine_moments / mhada_cosine_attn (linear cosine activation), mhada_warp_bwd; 13: mhada_clock_probe, knob wino4, knobs of removed variants dropped (attn_sched, wino_ws, wino_l2pf, gemm_f32b, gemm_n64_pp, gemm_n64_cen), attn_waves 0 = auto; 12: mhada_feat_stats; 10-12 also added a trailing relu_mask / relu argument to mhada_conv3x3_wino, mhada_reflect_fold and mhada_feat_loss_bwd and mhada_gemm relu = 2; 11: mhada_transpose64; 10: mhada_attn_train_fwd_vt; 9: 3-channel conv adjoints; 8: feat_loss_bwd; 7: gemm c2 / vt outputs, instnorm / attention backward helpers; 6: LayerNorm / pos-embed adjoints; 5: Winograd conv; 4: CONV3X3_ZERO, gemm_tn, backward helpers

extern "C" const char* mhada_last_error(void) { return mhada::g_last_error.c_str(); }

extern "C" int mhada_set_tuning(const char* name, int value) {
  using namespace mhada;
  read_env_once();
  if (!name) return fail("mhada_set_tuning: null name");
  for (const Knob& k : kKnobs) {
    if (!strcmp(k.name, name)) {
      if (!valid(name, value)) return fail(std::string("mhada_set_tuning: bad value for ") + name);
      g_tuning.*k.field = value;
      return MHADA_OK;
    }
  }
  return fail(std::string("mhada_set_tuning: unknown knob ") + name);
}

extern "C" int mhada_get_tuning(const char* name, int* value) {
  using namespace mhada;
  read_env_once();
  if (!name || !value) return fail("mhada_get_tuning: null argument");
  for (const Knob& k : kKnobs) {
    if (!strcmp(k.name, name)) {
      *value = g_tuning.*k.field;
      return MHADA_OK;
    }
  }
  return fail(std::string("mhada_get_tuning: unknown knob ") + name);
}
