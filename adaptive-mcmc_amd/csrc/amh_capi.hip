// amh_capi.hip -- the extern "C" boundary of libamh.so (include/amh.h).
// Validates arguments, keeps per-handle configuration and model binding, and
// enqueues the kernels of amh_kernels.hip on the caller's stream.
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "../../include/amh.h"
#include "../../include/amh_math.h"
#include "amh_internal.h"

#include <vector>

struct amh_handle {
  amh_config cfg;
  int device = 0;
  int model_id = 0;
  amh::ModelArgs model{nullptr, 0, 0};
  int64_t n_data = 0;
  float* gamma_tab = nullptr;  // device, kGammaTab entries
  double* partials = nullptr;  // pooled mode: chunk partial sums (scratch)
  size_t partials_bytes = 0;
  float* split_buf = nullptr;  // split path: proposals [C][d] then U(z') [C] (scratch)
  int64_t big_ready_C = -1;    // d > 64: split_buf holds the next proposal of the last output state (C chains)
  amh_state big_ready_out{};   // ... and that output state's buffers: READY is honoured only for these
  int64_t ext_ready_C = -1;    // external potential, d > 64: split_buf holds the solves (wa, wr, dg) of
  amh_state ext_ready_in{};    // the proposals formed from this state (amh_propose / amh_step_external)
  size_t split_bytes = 0;
  float* upd_buf = nullptr;    // pooled d > 64: Sigma' / L' staging (4-row-aligned layout) + ok flag
  size_t upd_bytes = 0;
  float* xpack = nullptr;      // diamonds: design matrix in MFMA tile order (made by amh_bind_model)
  float* noise_buf = nullptr;  // pooled d > 64: [cap] records (i, key0, key1, u bits) then xi [cap][d]
  size_t noise_bytes = 0;
  int64_t noise_cap = 0;       // chains the noise buffer holds
  int64_t noise_C = 0;         // chains of the last stats call, whose keys are at noise_keys
  const uint32_t* noise_keys = nullptr;
  int* err_host = nullptr;     // pooled d = 64: host-mapped device error flag (PooledUpdateParams::err_flag)
  int* err_dev = nullptr;      // ... its device address
  std::string err;
};

namespace {

thread_local std::string g_err;

int fail(amh_handle* h, int code, const std::string& msg) {
  if (h) h->err = msg; else g_err = msg;
  return code;
}

int hip_fail(amh_handle* h, hipError_t e, const char* where) {
  return fail(h, AMH_EHIP, std::string(where) + ": " + hipGetErrorString(e));
}

const char* const kUpdateStuck =
    "amh_pooled_update (d = 64): a factoring wave's bounded wait for an earlier wave's columns ran out in an "
    "earlier launch; that update kept the factor and covariance (the run no longer follows the bit spec)";

// a device-side failure flagged by an earlier (asynchronous) launch: reported
// by the handle's next pooled call and by amh_last_error, then cleared
int check_device_flag(amh_handle* h) {
  if (h && h->err_host && *(volatile int*)h->err_host != 0) {
    *(volatile int*)h->err_host = 0;
    return fail(h, AMH_EHIP, kUpdateStuck);
  }
  return AMH_OK;
}

bool same_buffers(const amh_state& a, const amh_state& b) {
  return a.i == b.i && a.z == b.z && a.potential_energy == b.potential_energy &&
         a.mean_accept_prob == b.mean_accept_prob && a.loc == b.loc && a.scale == b.scale &&
         a.log_step_size == b.log_step_size && a.as_change == b.as_change && a.rng_key == b.rng_key;
}

bool state_ok(const amh_state* s) {
  return s && s->i && s->z && s->potential_energy && s->mean_accept_prob && s->loc && s->scale &&
         s->log_step_size && s->as_change && s->rng_key;
}

int expected_dim(int model_id, int64_t n_data, const int64_t* ip, int nip, int d, std::string* why) {
  switch (model_id) {
    case AMH_MODEL_GAUSSIAN:
      if (n_data != (int64_t)d + (int64_t)d * d + 1) { *why = "gaussian data must hold d + d*d + 1 floats"; return -1; }
      return d;
    case AMH_MODEL_EIGHT_SCHOOLS: {
      if (nip < 1) { *why = "eight_schools needs iparams {J}"; return -1; }
      const int64_t J = ip[0];
      if (n_data != 3 * J) { *why = "eight_schools data must hold 3*J floats"; return -1; }
      return (int)(J + 2);
    }
    case AMH_MODEL_KIDIQ: {
      if (nip < 1) { *why = "kidiq needs iparams {N}"; return -1; }
      if (n_data != 3 * ip[0]) { *why = "kidiq data must hold 3*N floats"; return -1; }
      return 4;
    }
    case AMH_MODEL_DIAMONDS: {
      if (nip < 2) { *why = "diamonds needs iparams {N, K}"; return -1; }
      const int64_t N = ip[0], K = ip[1];
      if (n_data != N * (K - 1) + N) { *why = "diamonds data must hold N*(K-1) + N floats"; return -1; }
      return (int)(K + 1);
    }
    case AMH_MODEL_DIAMONDS_SS: {
      if (nip < 2) { *why = "diamonds_suffstat needs iparams {N, K}"; return -1; }
      const int64_t Kc = ip[1] - 1;
      if (Kc < 1 || Kc > 30) { *why = "diamonds_suffstat needs 2 <= K <= 31"; return -1; }
      if (n_data != 2 * (4 + 2 * Kc + Kc * Kc)) { *why = "diamonds_suffstat data must hold 2 (4 + 2 Kc + Kc^2) floats"; return -1; }
      return (int)(Kc + 2);
    }
    case AMH_MODEL_MIXTURE: {
      if (nip < 1) { *why = "mixture needs iparams {K}"; return -1; }
      if (ip[0] < 1 || ip[0] > 8) { *why = "mixture needs 1 <= K <= 8 components"; return -1; }
      if (n_data != 3 * ip[0]) { *why = "mixture data must hold 3*K floats"; return -1; }
      if (d < 1 || d > 16) { *why = "mixture needs 1 <= d <= 16"; return -1; }
      return d;
    }
    case AMH_MODEL_EXTERNAL:
      if (n_data < 0 || nip != 0) { *why = "external potential takes no data or iparams"; return -1; }
      if (d < 1 || d > 256) { *why = "external potential needs 1 <= d <= 256"; return -1; }
      return d;
    default:
      *why = "unknown model id";
      return -1;
  }
}

// device scratch of at least `need` bytes (grown, never shrunk); a queued
// launch may still read the old buffer, so the stream drains before the free
int grow(amh_handle* h, float** buf, size_t* have, size_t need, void* stream, const char* where) {
  if (need <= *have) return AMH_OK;
  if (*buf) {
    (void)hipStreamSynchronize((hipStream_t)stream);
    (void)hipFree(*buf);
  }
  *buf = nullptr;
  *have = 0;
  hipError_t e = hipMalloc(buf, need);
  if (e != hipSuccess) return hip_fail(h, e, where);
  *have = need;
  return AMH_OK;
}

}  // namespace

extern "C" {

int amh_version(void) { return AMH_ABI_VERSION; }

const char* amh_last_error(const amh_handle* h) {
  if (h && h->err_host && *(volatile int*)h->err_host != 0) const_cast<amh_handle*>(h)->err = kUpdateStuck;
  return h ? h->err.c_str() : g_err.c_str();
}

int amh_create(const amh_config* cfg, int device, amh_handle** out) {
  if (!cfg || !out) return fail(nullptr, AMH_EINVAL, "amh_create: null argument");
  if (cfg->dim < 1 || cfg->dim > 256) return fail(nullptr, AMH_EINVAL, "amh_create: dim must be in [1, 256]");
  if (cfg->num_warmup < 0) return fail(nullptr, AMH_EINVAL, "amh_create: num_warmup < 0");
  amh_handle* h = new (std::nothrow) amh_handle();
  if (!h) return fail(nullptr, AMH_ENOMEM, "amh_create: out of memory");
  h->cfg = *cfg;
  h->device = device;
  // gamma_n = 1 / n^a for n < kGammaTab, evaluated on the host by the same
  // routine the kernels use for larger n (include/amh_math.h).
  std::vector<float> tab(amh::kGammaTab);
  tab[0] = 1.0f;
  for (int32_t n = 1; n < amh::kGammaTab; ++n) tab[n] = amh_lr_gamma(n, cfg->lr_decay);
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc(&h->gamma_tab, sizeof(float) * tab.size());
  if (e == hipSuccess) e = hipMemcpy(h->gamma_tab, tab.data(), sizeof(float) * tab.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    const int rc = hip_fail(nullptr, e, "amh_create");
    if (h->gamma_tab) (void)hipFree(h->gamma_tab);
    delete h;
    return rc;
  }
  *out = h;
  return AMH_OK;
}

int amh_check_device(amh_handle* h) {
  if (!h) return fail(nullptr, AMH_EINVAL, "amh_check_device: null handle");
  return check_device_flag(h);
}

int amh_destroy(amh_handle* h) {
  int rc = AMH_OK;
  if (h) {
    (void)hipSetDevice(h->device);
    // no device-wide synchronisation here (destroy runs from
    // finalisers): the flag is read as it stands; a launch still in flight is
    // covered by amh_check_device after the caller synchronised its stream.
    // hipFree below orders the frees after outstanding work as HIP defines.
    if (h->err_host && *(volatile int*)h->err_host != 0) rc = fail(nullptr, AMH_EHIP, kUpdateStuck);
    if (h->gamma_tab) (void)hipFree(h->gamma_tab);
    if (h->partials) (void)hipFree(h->partials);
    if (h->split_buf) (void)hipFree(h->split_buf);
    if (h->upd_buf) (void)hipFree(h->upd_buf);
    if (h->xpack) (void)hipFree(h->xpack);
    if (h->noise_buf) (void)hipFree(h->noise_buf);
    if (h->err_host) (void)hipHostFree(h->err_host);
  }
  delete h;
  return rc;
}

int amh_bind_model(amh_handle* h, int32_t model_id, const float* data, int64_t n_data, const int64_t* iparams,
                   int32_t n_iparams) {
  if (!h) return fail(nullptr, AMH_EINVAL, "amh_bind_model: null handle");
  if (!data) return fail(h, AMH_EINVAL, "amh_bind_model: null data");
  std::string why;
  const int dm = expected_dim(model_id, n_data, iparams, n_iparams, h->cfg.dim, &why);
  if (dm < 0) return fail(h, AMH_EINVAL, "amh_bind_model: " + why);
  if (dm != h->cfg.dim)
    return fail(h, AMH_EINVAL, "amh_bind_model: model dimension " + std::to_string(dm) + " != config dim " +
                                   std::to_string(h->cfg.dim));
  if (dm > 64 && !amh::big_model(model_id, dm) && model_id != AMH_MODEL_EXTERNAL)
    return fail(h, AMH_EINVAL, "amh_bind_model: d > 64 needs the Gaussian model or an external potential (d <= 256)");
  // the handle's device for everything below (the caller -- Handle.bind_model --
  // holds it current and restores its own afterwards)
  hipError_t e = hipSetDevice(h->device);
  if (e != hipSuccess) return hip_fail(h, e, "amh_bind_model/hipSetDevice");
  if (h->xpack) {
    (void)hipDeviceSynchronize();  // a queued launch may still read the old copy
    (void)hipFree(h->xpack);
    h->xpack = nullptr;
  }
  h->model_id = 0;  // unbound until the whole binding has succeeded
  h->model.data = data;
  const bool dia = model_id == AMH_MODEL_DIAMONDS || model_id == AMH_MODEL_DIAMONDS_SS;
  h->model.n = (model_id == AMH_MODEL_KIDIQ || model_id == AMH_MODEL_MIXTURE || dia) ? iparams[0] : 0;
  h->model.k = dia ? iparams[1] : 0;
  h->n_data = n_data;
  if (model_id == AMH_MODEL_DIAMONDS && amh::split_model(model_id, dm)) {
    // the MFMA potential's tile copy of Xc and Y, made once here (synchronous,
    // on the null stream: the caller has synchronised the stream that wrote data)
    const int64_t nf = amh::diamonds_pack_floats(h->model.n, h->model.k);
    if (nf > 0) {
      e = hipMalloc(&h->xpack, (size_t)nf * sizeof(float));
      if (e == hipSuccess) e = amh::run_diamonds_pack(h->model, h->xpack, nullptr);
      if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
      if (e != hipSuccess) {
        if (h->xpack) (void)hipFree(h->xpack);
        h->xpack = nullptr;
        return hip_fail(h, e, "amh_bind_model(diamonds tile copy)");
      }
    }
  }
  h->model_id = model_id;
  return AMH_OK;
}

int amh_init(amh_handle* h, const uint32_t key[2], int64_t chain_offset, int64_t num_chains, const float* init_z,
             const amh_state* out, void* stream) {
  if (!h) return fail(nullptr, AMH_EINVAL, "amh_init: null handle");
  if (!h->model_id) return fail(h, AMH_ENOMODEL, "amh_init: no model bound");
  if (!key || !state_ok(out) || num_chains < 1 || chain_offset < 0)
    return fail(h, AMH_EINVAL, "amh_init: bad arguments");
  h->big_ready_C = -1;  // a kept proposal belongs to a state this call may overwrite
  h->ext_ready_C = -1;
  hipError_t e = hipSetDevice(h->device);
  if (e != hipSuccess) return hip_fail(h, e, "amh_init/hipSetDevice");
  amh::InitParams p{};
  p.out = *out;
  p.C = num_chains;
  p.chain_offset = chain_offset;
  p.d = h->cfg.dim;
  p.key0 = key[0];
  p.key1 = key[1];
  p.init_z = init_z;
  p.model = h->model;
  if (h->model_id == AMH_MODEL_EXTERNAL && p.d > 64) {
    e = amh::run_big_init(p, (hipStream_t)stream);  // pe0 = 0: the caller evaluates U(z0)
  } else if (amh::big_model(h->model_id, p.d)) {
    e = amh::run_big_init(p, (hipStream_t)stream);
    if (e == hipSuccess) {
      amh::PotParams q{out->z, out->potential_energy, num_chains, p.d, h->model};
      e = amh::run_big_potential(q, (hipStream_t)stream);
    }
  } else if (h->model_id == AMH_MODEL_EXTERNAL) {
    e = amh::run_init_nopot(p, (hipStream_t)stream);  // pe0 = 0: the caller evaluates U(z0)
  } else if (amh::split_model(h->model_id, p.d)) {
    // pe0 = U(z0) from the lane-per-chain potential (bit-identical to the group one)
    e = amh::run_init_nopot(p, (hipStream_t)stream);
    if (e == hipSuccess) {
      amh::PotParams q{out->z, out->potential_energy, num_chains, p.d, h->model, h->xpack};
      e = amh::run_potential_lane(h->model_id, q, (hipStream_t)stream);
    }
  } else {
    e = amh::run_init(h->model_id, p, (hipStream_t)stream);
  }
  if (e != hipSuccess) return hip_fail(h, e, "amh_init");
  return AMH_OK;
}

int amh_step(amh_handle* h, int64_t num_chains, const amh_state* in, const amh_state* out, int32_t n_steps,
             const amh_collect* collect, void* stream) {
  return amh_step_chained(h, num_chains, in, out, n_steps, collect, 0, stream);
}

int amh_step_chained(amh_handle* h, int64_t num_chains, const amh_state* in, const amh_state* out,
                     int32_t n_steps, const amh_collect* collect, int32_t flags, void* stream) {
  if (!h) return fail(nullptr, AMH_EINVAL, "amh_step: null handle");
  if (!h->model_id) return fail(h, AMH_ENOMODEL, "amh_step: no model bound");
  if (!state_ok(in) || !state_ok(out) || num_chains < 1 || n_steps < 0)
    return fail(h, AMH_EINVAL, "amh_step: bad arguments");
  if (h->model_id == AMH_MODEL_EXTERNAL)
    return fail(h, AMH_EINVAL, "amh_step: an external potential runs through amh_propose / amh_step_external");
  if (n_steps == 0) {
    h->big_ready_C = -1;  // a kept proposal never survives a call it was not used in
    return AMH_OK;
  }
  if (collect && collect->thinning < 1) return fail(h, AMH_EINVAL, "amh_step: thinning must be >= 1");
  hipError_t e = hipSetDevice(h->device);
  if (e != hipSuccess) return hip_fail(h, e, "amh_step/hipSetDevice");
  amh::StepParams p{};
  p.in = *in;
  p.out = *out;
  p.C = num_chains;
  p.d = h->cfg.dim;
  p.W = h->cfg.num_warmup;
  p.a = h->cfg.lr_decay;
  p.target = h->cfg.target_accept_prob;
  p.eps = h->cfg.eps;
  p.n_steps = n_steps;
  p.thinning = collect ? collect->thinning : 1;
  p.col_z = collect ? collect->z : nullptr;
  p.col_pe = collect ? collect->potential_energy : nullptr;
  p.accept_count = collect ? collect->accept_count : nullptr;
  p.gamma_tab = h->gamma_tab;
  p.gamma_tab_n = amh::kGammaTab;
  p.model = h->model;
  if (amh::big_model(h->model_id, p.d)) {
    // d > 64: propose pass, MFMA potential, step pass per transition
    const int64_t C = num_chains;
    const size_t need = (size_t)C * (size_t)(4 * p.d + 1) * sizeof(float);
    int rc = grow(h, &h->split_buf, &h->split_bytes, need, stream, "amh_step/hipMalloc");
    if (rc != AMH_OK) return rc;
    amh::BigParams q{};
    q.out = *out;
    q.C = C;
    q.d = p.d;
    q.W = p.W;
    q.a = p.a;
    q.target = p.target;
    q.eps = p.eps;
    q.gamma_tab = p.gamma_tab;
    q.gamma_tab_n = p.gamma_tab_n;
    q.xprop = h->split_buf;
    q.wa = q.xprop + (size_t)C * p.d;
    q.wr = q.wa + (size_t)C * p.d;
    q.dg = q.wr + (size_t)C * p.d;
    float* pep = q.dg + (size_t)C * p.d;
    q.pep = pep;
    q.accept_count = p.accept_count;
    // the caller vouches (AMH_STEP_PROPOSAL_READY) that `in` is the unchanged
    // output of the previous call, which kept its next proposal in the scratch
    // (and `in` must be the very buffers that call wrote)
    const bool ready = (flags & AMH_STEP_PROPOSAL_READY) && h->big_ready_C == C && same_buffers(*in, h->big_ready_out);
    const bool keep_next = (flags & AMH_STEP_KEEP_PROPOSAL) != 0;
    h->big_ready_C = -1;
    for (int32_t t = 0; t < n_steps; ++t) {
      q.in = (t == 0) ? *in : *out;
      const bool keep = ((t + 1) % p.thinning) == 0;
      const int64_t k = t / p.thinning;
      q.col_z = (keep && p.col_z) ? p.col_z + (size_t)k * C * p.d : nullptr;
      q.col_pe = (keep && p.col_pe) ? p.col_pe + (size_t)k * C : nullptr;
      // the first transition's proposal comes from the propose pass (or the
      // previous call); each step pass forms the next one on the fly, so the
      // factor is read once per transition
      if (t == 0 && !ready) e = amh::run_big_propose(q, (hipStream_t)stream);
      if (e == hipSuccess) {
        amh::PotParams pp{q.xprop, pep, C, p.d, h->model};
        e = amh::run_big_potential(pp, (hipStream_t)stream);
      }
      if (e == hipSuccess) e = amh::run_big_step(q, (hipStream_t)stream, t + 1 < n_steps || keep_next);
      if (e != hipSuccess) return hip_fail(h, e, "amh_step(d > 64)");
    }
    h->big_ready_C = keep_next ? C : -1;
    h->big_ready_out = *out;
    return AMH_OK;
  }
  if (amh::split_model(h->model_id, p.d)) {
    // one transition = propose, batched potential, step(U(z') from memory);
    // collection is per launch: step t keeps slot t / thinning when (t+1) % thinning == 0
    const int64_t C = num_chains;
    const size_t need = (size_t)C * (size_t)(p.d + 1) * sizeof(float);
    const bool grown = need > h->split_bytes;
    int rc = grow(h, &h->split_buf, &h->split_bytes, need, stream, "amh_step/hipMalloc");
    if (rc != AMH_OK) return rc;
    // READY / KEEP as for d > 64: the step pass of each transition forms the
    // next one's proposal (so the factor is read once per transition); only
    // the first transition of a call may need the propose pass
    const bool ready = !grown && (flags & AMH_STEP_PROPOSAL_READY) && h->big_ready_C == C &&
                       same_buffers(*in, h->big_ready_out);
    const bool keep_next = (flags & AMH_STEP_KEEP_PROPOSAL) != 0;
    h->big_ready_C = -1;
    float* xprop = h->split_buf;
    float* peprop = h->split_buf + (size_t)C * p.d;
    amh::StepParams q = p;
    q.n_steps = 1;
    q.thinning = 1;
    q.ext_pe = peprop;
    q.ext_z = xprop;
    for (int32_t t = 0; t < n_steps; ++t) {
      q.in = (t == 0) ? *in : *out;
      const bool keep = ((t + 1) % p.thinning) == 0;
      const int64_t k = t / p.thinning;
      q.col_z = (keep && p.col_z) ? p.col_z + (size_t)k * C * p.d : nullptr;
      q.col_pe = (keep && p.col_pe) ? p.col_pe + (size_t)k * C : nullptr;
      q.xprop_next = (t + 1 < n_steps || keep_next) ? xprop : nullptr;
      if (t == 0 && !ready) e = amh::run_propose(q, xprop, (hipStream_t)stream);
      if (e == hipSuccess) {
        amh::PotParams pp{xprop, peprop, C, p.d, h->model, h->xpack};
        e = amh::run_potential_lane(h->model_id, pp, (hipStream_t)stream);
      }
      if (e == hipSuccess) e = amh::run_step_ext(q, (hipStream_t)stream);
      if (e != hipSuccess) return hip_fail(h, e, "amh_step(split)");
    }
    h->big_ready_C = keep_next ? C : -1;
    h->big_ready_out = *out;
    return AMH_OK;
  }
  e = amh::run_step(h->model_id, p, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(h, e, "amh_step");
  return AMH_OK;
}

int amh_potential(amh_handle* h, const float* z, float* pe, int64_t n, void* stream) {
  if (!h) return fail(nullptr, AMH_EINVAL, "amh_potential: null handle");
  if (!h->model_id) return fail(h, AMH_ENOMODEL, "amh_potential: no model bound");
  if (!z || !pe || n < 1) return fail(h, AMH_EINVAL, "amh_potential: bad arguments");
  if (h->model_id == AMH_MODEL_EXTERNAL) return fail(h, AMH_EINVAL, "amh_potential: the potential is external");
  hipError_t e = hipSetDevice(h->device);
  if (e != hipSuccess) return hip_fail(h, e, "amh_potential/hipSetDevice");
  amh::PotParams p{z, pe, n, h->cfg.dim, h->model, h->xpack};
  e = amh::big_model(h->model_id, p.d)     ? amh::run_big_potential(p, (hipStream_t)stream)
      : amh::split_model(h->model_id, p.d) ? amh::run_potential_lane(h->model_id, p, (hipStream_t)stream)
                                           : amh::run_potential(h->model_id, p, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(h, e, "amh_potential");
  return AMH_OK;
}

// ------------------------------------------------- external potential --
// AMH_MODEL_EXTERNAL: the split transition (amh_split.hip propose_kernel,
// the step kernel with U(z') read from memory -- the diamonds path's two
// launches) with the caller's U in between.
static amh::StepParams ext_params(amh_handle* h, int64_t C, const amh_state* in, const amh_state* out) {
  amh::StepParams p{};
  p.in = *in;
  p.out = *out;
  p.C = C;
  p.d = h->cfg.dim;
  p.W = h->cfg.num_warmup;
  p.a = h->cfg.lr_decay;
  p.target = h->cfg.target_accept_prob;
  p.eps = h->cfg.eps;
  p.n_steps = 1;
  p.thinning = 1;
  p.gamma_tab = h->gamma_tab;
  p.gamma_tab_n = amh::kGammaTab;
  p.model = h->model;
  return p;
}

// d > 64: big_propose_kernel / big_step_kernel with the caller's U(z'); the
// proposals live in the caller's zprop, the solves (wa, wr) and the diagonal
// in the handle's scratch, tied to the state they were formed from
static int ext_big_params(amh_handle* h, int64_t C, const amh_state* in, const amh_state* out, float* zprop,
                          void* stream, amh::BigParams* q) {
  const int d = h->cfg.dim;
  const size_t need = (size_t)C * (size_t)(3 * d) * sizeof(float);
  const bool grown = need > h->split_bytes;
  int rc = grow(h, &h->split_buf, &h->split_bytes, need, stream, "amh_propose/hipMalloc");
  if (rc != AMH_OK) return rc;
  if (grown) h->ext_ready_C = -1;
  h->big_ready_C = -1;  // the scratch now holds the external path's solves
  *q = amh::BigParams{};
  q->in = *in;
  q->out = *out;
  q->C = C;
  q->d = d;
  q->W = h->cfg.num_warmup;
  q->a = h->cfg.lr_decay;
  q->target = h->cfg.target_accept_prob;
  q->eps = h->cfg.eps;
  q->gamma_tab = h->gamma_tab;
  q->gamma_tab_n = amh::kGammaTab;
  q->xprop = zprop;
  q->wa = h->split_buf;
  q->wr = q->wa + (size_t)C * d;
  q->dg = q->wr + (size_t)C * d;
  return AMH_OK;
}

int amh_propose(amh_handle* h, int64_t num_chains, const amh_state* in, float* zprop, void* stream) {
  if (!h) return fail(nullptr, AMH_EINVAL, "amh_propose: null handle");
  if (h->model_id != AMH_MODEL_EXTERNAL) return fail(h, AMH_EINVAL, "amh_propose: needs AMH_MODEL_EXTERNAL");
  if (!state_ok(in) || !zprop || num_chains < 1) return fail(h, AMH_EINVAL, "amh_propose: bad arguments");
  hipError_t e = hipSetDevice(h->device);
  if (e != hipSuccess) return hip_fail(h, e, "amh_propose/hipSetDevice");
  if (h->cfg.dim > 64) {
    amh::BigParams q;
    int rc = ext_big_params(h, num_chains, in, in, zprop, stream, &q);
    if (rc != AMH_OK) return rc;
    e = amh::run_big_propose(q, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(h, e, "amh_propose(d > 64)");
    h->ext_ready_C = num_chains;
    h->ext_ready_in = *in;
    return AMH_OK;
  }
  const amh::StepParams p = ext_params(h, num_chains, in, in);
  e = amh::run_propose(p, zprop, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(h, e, "amh_propose");
  return AMH_OK;
}

int amh_step_external(amh_handle* h, int64_t num_chains, const amh_state* in, const amh_state* out,
                      const float* zprop, const float* pe_prop, float* zprop_next, const amh_collect* collect,
                      void* stream) {
  if (!h) return fail(nullptr, AMH_EINVAL, "amh_step_external: null handle");
  if (h->model_id != AMH_MODEL_EXTERNAL)
    return fail(h, AMH_EINVAL, "amh_step_external: needs AMH_MODEL_EXTERNAL");
  if (!state_ok(in) || !state_ok(out) || !zprop || !pe_prop || num_chains < 1)
    return fail(h, AMH_EINVAL, "amh_step_external: bad arguments");
  if (collect && collect->thinning != 1) return fail(h, AMH_EINVAL, "amh_step_external: thinning must be 1");
  hipError_t e = hipSetDevice(h->device);
  if (e != hipSuccess) return hip_fail(h, e, "amh_step_external/hipSetDevice");
  if (h->cfg.dim > 64) {
    // the step pass reads the solves amh_propose (or the previous step) formed
    // for exactly this state, and writes the next proposals in place
    if (h->ext_ready_C != num_chains || !same_buffers(*in, h->ext_ready_in))
      return fail(h, AMH_EINVAL, "amh_step_external: d > 64 needs the proposals of this state (amh_propose first)");
    if (zprop_next && zprop_next != zprop)
      return fail(h, AMH_EINVAL, "amh_step_external: d > 64 forms the next proposals in place (zprop_next == zprop)");
    amh::BigParams q;
    int rc = ext_big_params(h, num_chains, in, out, const_cast<float*>(zprop), stream, &q);
    if (rc != AMH_OK) return rc;
    q.pep = pe_prop;
    q.accept_count = collect ? collect->accept_count : nullptr;
    q.col_z = collect ? collect->z : nullptr;
    q.col_pe = collect ? collect->potential_energy : nullptr;
    h->ext_ready_C = -1;
    e = amh::run_big_step(q, (hipStream_t)stream, zprop_next != nullptr);
    if (e != hipSuccess) return hip_fail(h, e, "amh_step_external(d > 64)");
    if (zprop_next) {
      h->ext_ready_C = num_chains;
      h->ext_ready_in = *out;
    }
    return AMH_OK;
  }
  amh::StepParams p = ext_params(h, num_chains, in, out);
  p.col_z = collect ? collect->z : nullptr;
  p.col_pe = collect ? collect->potential_energy : nullptr;
  p.accept_count = collect ? collect->accept_count : nullptr;
  p.ext_z = zprop;
  p.ext_pe = pe_prop;
  p.xprop_next = zprop_next;
  e = amh::run_step_ext(p, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(h, e, "amh_step_external");
  return AMH_OK;
}

static int pnx_ext(amh_handle* h, const uint32_t key[2], float* z, float* pe, int64_t C, const float* scale,
                   float lam, int32_t t, float* zprop, const float* pe_prop, bool accept, void* stream,
                   const char* who) {
  if (!h) return fail(nullptr, AMH_EINVAL, std::string(who) + ": null handle");
  if (h->model_id != AMH_MODEL_EXTERNAL) return fail(h, AMH_EINVAL, std::string(who) + ": needs AMH_MODEL_EXTERNAL");
  if (h->cfg.dim > 64) return fail(h, AMH_EINVAL, std::string(who) + ": an external sample_Pnx needs d <= 64");
  if (!key || !z || !zprop || C < 1 || t < 0 || (accept ? (!pe || !pe_prop) : !scale))
    return fail(h, AMH_EINVAL, std::string(who) + ": bad arguments");
  hipError_t e = hipSetDevice(h->device);
  if (e != hipSuccess) return hip_fail(h, e, (std::string(who) + "/hipSetDevice").c_str());
  amh::PnxExtParams p{};
  p.z = z;
  p.pe = pe;
  p.zprop = zprop;
  p.pe_prop = pe_prop;
  p.C = C;
  p.scale = scale;
  p.log_step_size = lam;
  p.eps = h->cfg.eps;
  p.t = t;
  p.d = h->cfg.dim;
  p.key0 = key[0];
  p.key1 = key[1];
  e = amh::run_pnx_ext(p, accept, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(h, e, who);
  return AMH_OK;
}

int amh_pnx_propose(amh_handle* h, const uint32_t key[2], const float* z, int64_t num_chains,
                    const float* scale_packed, float log_step_size, int32_t t, float* zprop, void* stream) {
  return pnx_ext(h, key, const_cast<float*>(z), nullptr, num_chains, scale_packed, log_step_size, t, zprop, nullptr,
                 false, stream, "amh_pnx_propose");
}

int amh_pnx_accept(amh_handle* h, const uint32_t key[2], float* z, float* pe, int64_t num_chains,
                   const float* zprop, const float* pe_prop, int32_t t, void* stream) {
  return pnx_ext(h, key, z, pe, num_chains, nullptr, 0.0f, t, const_cast<float*>(zprop), pe_prop, true, stream,
                 "amh_pnx_accept");
}

int amh_sample_pnx(amh_handle* h, const uint32_t key[2], const float* x, int64_t n_points, int64_t n_samples,
                   const float* loc, const float* scale_packed, float log_step_size, int32_t n, float* out,
                   void* stream) {
  (void)loc;  // the frozen kernel's proposal does not read the mean (arwmh.py:166-167)
  if (!h) return fail(nullptr, AMH_EINVAL, "amh_sample_pnx: null handle");
  if (!h->model_id) return fail(h, AMH_ENOMODEL, "amh_sample_pnx: no model bound");
  if (!key || !x || !scale_packed || !out || n_points < 1 || n_samples < 1 || n < 0)
    return fail(h, AMH_EINVAL, "amh_sample_pnx: bad arguments");
  if (h->cfg.dim > 64 && !amh::big_model(h->model_id, h->cfg.dim))
    return fail(h, AMH_EINVAL, "amh_sample_pnx: d > 64 needs the dense Gaussian (d <= 256)");
  if (h->model_id == AMH_MODEL_EXTERNAL)
    return fail(h, AMH_EINVAL, "amh_sample_pnx: an external potential runs through amh_pnx_propose / amh_pnx_accept");
  hipError_t e = hipSetDevice(h->device);
  if (e != hipSuccess) return hip_fail(h, e, "amh_sample_pnx/hipSetDevice");
  amh::PnxParams p{};
  p.x = x;
  p.n_points = n_points;
  p.n_samples = n_samples;
  p.scale = scale_packed;
  p.log_step_size = log_step_size;
  p.eps = h->cfg.eps;
  p.n = n;
  p.d = h->cfg.dim;
  p.key0 = key[0];
  p.key1 = key[1];
  p.out = out;
  p.model = h->model;
  e = (p.d > 64) ? amh::run_big_pnx(p, (hipStream_t)stream) : amh::run_pnx(h->model_id, p, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(h, e, "amh_sample_pnx");
  return AMH_OK;
}

int amh_chain_keys(const uint32_t key[2], int64_t chain_offset, int64_t n, uint32_t* out, void* stream) {
  if (!key || !out || n < 1 || chain_offset < 0) return fail(nullptr, AMH_EINVAL, "amh_chain_keys: bad arguments");
  hipError_t e = amh::run_chain_keys(key[0], key[1], chain_offset, n, out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(nullptr, e, "amh_chain_keys");
  return AMH_OK;
}

// -------------------------------------------------------------------- ASSS --
static bool asss_state_ok(const amh_state* s) {
  return s && s->i && s->z && s->potential_energy && s->loc && s->scale && s->as_change && s->rng_key;
}

int amh_asss_step(amh_handle* h, int64_t num_chains, const amh_state* in, const amh_state* out, int32_t n_steps,
                  const amh_collect* collect, void* stream) {
  if (!h) return fail(nullptr, AMH_EINVAL, "amh_asss_step: null handle");
  if (!h->model_id) return fail(h, AMH_ENOMODEL, "amh_asss_step: no model bound");
  if (!asss_state_ok(in) || !asss_state_ok(out) || num_chains < 1 || n_steps < 0)
    return fail(h, AMH_EINVAL, "amh_asss_step: bad arguments");
  const bool big = amh::big_model(h->model_id, h->cfg.dim);
  if (h->cfg.dim > 64 && !big)
    return fail(h, AMH_EINVAL, "amh_asss_step: dim must be <= 64, or a dense Gaussian up to 256");
  if (h->model_id == AMH_MODEL_EXTERNAL)
    return fail(h, AMH_EINVAL, "amh_asss_step: the slice sampler needs a device potential (not external)");
  if (collect && collect->thinning < 1) return fail(h, AMH_EINVAL, "amh_asss_step: thinning must be >= 1");
  if (n_steps == 0) return AMH_OK;
  hipError_t e = hipSetDevice(h->device);
  if (e != hipSuccess) return hip_fail(h, e, "amh_asss_step/hipSetDevice");
  amh::StepParams p{};
  p.in = *in;
  p.out = *out;
  p.C = num_chains;
  p.d = h->cfg.dim;
  p.W = h->cfg.num_warmup;
  p.a = h->cfg.lr_decay;
  p.target = h->cfg.target_accept_prob;
  p.eps = h->cfg.eps;
  p.n_steps = n_steps;
  p.thinning = collect ? collect->thinning : 1;
  p.col_z = collect ? collect->z : nullptr;
  p.col_pe = collect ? collect->potential_energy : nullptr;
  p.accept_count = nullptr;
  p.gamma_tab = h->gamma_tab;
  p.gamma_tab_n = amh::kGammaTab;
  p.model = h->model;
  if (big) {
    // large d: one launch per transition (the factor streamed four times),
    // the first from `in`, the rest in place on `out`
    const int64_t keep_stride = num_chains * (int64_t)h->cfg.dim;
    for (int32_t t = 0; t < n_steps; ++t) {
      amh::StepParams q = p;
      if (t > 0) q.in = *out;
      q.n_steps = 1;
      const bool keep = (t + 1) % p.thinning == 0;
      const int64_t k = (t + 1) / p.thinning - 1;
      q.col_z = (keep && p.col_z) ? p.col_z + k * keep_stride : nullptr;
      q.col_pe = (keep && p.col_pe) ? p.col_pe + k * num_chains : nullptr;
      e = amh::run_asss_big_step(q, (hipStream_t)stream);
      if (e != hipSuccess) return hip_fail(h, e, "amh_asss_step(large d)");
    }
    return AMH_OK;
  }
  e = amh::run_asss_step(h->model_id, p, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(h, e, "amh_asss_step");
  return AMH_OK;
}

int amh_asss_sample_pnx(amh_handle* h, const uint32_t key[2], const float* x, int64_t n_points, int64_t n_samples,
                        const float* loc, const float* scale_packed, int32_t n, float* out, void* stream) {
  if (!h) return fail(nullptr, AMH_EINVAL, "amh_asss_sample_pnx: null handle");
  if (!h->model_id) return fail(h, AMH_ENOMODEL, "amh_asss_sample_pnx: no model bound");
  if (!key || !x || !loc || !scale_packed || !out || n_points < 1 || n_samples < 1 || n < 0)
    return fail(h, AMH_EINVAL, "amh_asss_sample_pnx: bad arguments");
  const bool big = amh::big_model(h->model_id, h->cfg.dim);
  if (h->cfg.dim > 64 && !big)
    return fail(h, AMH_EINVAL, "amh_asss_sample_pnx: dim must be <= 64, or a dense Gaussian up to 256");
  if (h->model_id == AMH_MODEL_EXTERNAL)
    return fail(h, AMH_EINVAL, "amh_asss_sample_pnx: the slice sampler needs a device potential (not external)");
  hipError_t e = hipSetDevice(h->device);
  if (e != hipSuccess) return hip_fail(h, e, "amh_asss_sample_pnx/hipSetDevice");
  amh::AsssPnxParams p{};
  p.x = x;
  p.n_points = n_points;
  p.n_samples = n_samples;
  p.loc = loc;
  p.scale = scale_packed;
  p.eps = h->cfg.eps;
  p.n = n;
  p.d = h->cfg.dim;
  p.key0 = key[0];
  p.key1 = key[1];
  p.out = out;
  p.model = h->model;
  e = big ? amh::run_asss_big_pnx(p, (hipStream_t)stream) : amh::run_asss_pnx(h->model_id, p, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(h, e, "amh_asss_sample_pnx");
  return AMH_OK;
}

// -------------------------------------------------------------- evaluation --
int64_t amh_kernel_sum_scratch(int64_t n, int64_t m) { return n > 0 && m > 0 ? amh::kernel_sum_blocks(n, m) : 0; }

int amh_kernel_sum(const float* a, int64_t n, const float* b, int64_t m, int32_t d, float gamma, int32_t skip_diag,
                   double* scratch, double* out, void* stream) {
  if (!a || !b || !scratch || !out || n < 1 || m < 1 || d < 1)
    return fail(nullptr, AMH_EINVAL, "amh_kernel_sum: bad arguments");
  const hipError_t e = amh::run_kernel_sum(a, n, b, m, d, gamma, skip_diag, scratch, out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(nullptr, e, "amh_kernel_sum");
  return AMH_OK;
}

int amh_pairwise_dist2(const float* a, int64_t n, const float* b, int64_t m, int32_t d, float* out, void* stream) {
  if (!a || !b || !out || n < 1 || m < 1 || d < 1) return fail(nullptr, AMH_EINVAL, "amh_pairwise_dist2: bad arguments");
  const hipError_t e = amh::run_dist2(a, n, b, m, d, out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(nullptr, e, "amh_pairwise_dist2");
  return AMH_OK;
}

int amh_sinkhorn_lse(const float* cost, int64_t rows, int64_t cols, const float* pot, float log_w, float eps,
                     float* out, void* stream) {
  if (!cost || !pot || !out || rows < 1 || cols < 1 || !(eps > 0.0f) || rows > 0x7FFFFFFF)
    return fail(nullptr, AMH_EINVAL, "amh_sinkhorn_lse: bad arguments");
  const hipError_t e = amh::run_lse_rows(cost, rows, cols, pot, log_w, eps, out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(nullptr, e, "amh_sinkhorn_lse");
  return AMH_OK;
}

int amh_normals(const uint32_t key[2], int64_t n, float* out, void* stream) {
  if (!key || !out || n < 0) return fail(nullptr, AMH_EINVAL, "amh_normals: bad arguments");
  if (n == 0) return AMH_OK;
  const hipError_t e = amh::run_normals(key[0], key[1], n, out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(nullptr, e, "amh_normals");
  return AMH_OK;
}

// ------------------------------------------------------- pooled covariance --
static bool pooled_ok(const amh_pooled_state* s) {
  return s && s->i && s->z && s->potential_energy && s->rng_key && s->mean_accept_prob && s->loc && s->scale &&
         s->log_step_size && s->as_change && s->cov;
}

int amh_pooled_sums_size(int32_t dim, int64_t* v) {
  if (dim < 1 || dim > 256 || !v) return fail(nullptr, AMH_EINVAL, "amh_pooled_sums_size: bad arguments");
  *v = (int64_t)dim + (int64_t)dim * (dim + 1) / 2 + 2;
  return AMH_OK;
}

}  // extern "C"

// prep_for_update: the update follows in the same library call with no
// exchange in between (amh_pooled_step_k on one rank), so the large-d
// reduction's last kernel also forms that update's Sigma'
// A/B switches of the diagnostic build only (-DAMH_DIAG, `make stamps`; the
// bits are the same either way, the release library reads no environment):
// AMH_POOLED_FUSED_REDUCE=0 keeps the d = 64 reduction in its own launch;
// AMH_POOLED_NOISE_AHEAD=0 draws no noise ahead (each stats kernel draws its own)
static bool reduce_fusion_off() {
#ifdef AMH_DIAG
  static const bool off = [] {
    const char* e = getenv("AMH_POOLED_FUSED_REDUCE");
    return e != nullptr && e[0] == '0';
  }();
  return off;
#else
  return false;
#endif
}

static bool noise_ahead_off() {
#ifdef AMH_DIAG
  static const bool off = [] {
    const char* e = getenv("AMH_POOLED_NOISE_AHEAD");
    return e != nullptr && e[0] == '0';
  }();
  return off;
#else
  return false;
#endif
}

// d = 64 with prep_for_update: the last step's chunk partials are left
// unreduced; *deferred describes them for the update launch, which reduces
// them first (one launch fewer per pooled block)
struct DeferredReduce {
  const float* partials = nullptr;
  int64_t n_chunks = 0;
  int32_t accumulate = 0;
};

static int pooled_stats_impl(amh_handle* h, int64_t num_chains, const amh_pooled_state* in, int32_t k_steps,
                             float* z_out, float* pe_out, double* sums, void* stream, bool prep_for_update,
                             bool* sigma_ready, DeferredReduce* deferred = nullptr, bool pack_ready = false) {
  if (sigma_ready) *sigma_ready = false;
  if (deferred) *deferred = DeferredReduce{};
  if (!h) return fail(nullptr, AMH_EINVAL, "amh_pooled_stats: null handle");
  if (!h->model_id) return fail(h, AMH_ENOMODEL, "amh_pooled_stats: no model bound");
  if (!pooled_ok(in) || !z_out || !pe_out || !sums || num_chains < 1 || k_steps < 1)
    return fail(h, AMH_EINVAL, "amh_pooled_stats: bad arguments");
  if (int rc = check_device_flag(h)) return rc;
  hipError_t e = hipSetDevice(h->device);
  if (e != hipSuccess) return hip_fail(h, e, "amh_pooled_stats/hipSetDevice");
  const int d = h->cfg.dim;
  const bool big = amh::pooled_big_model(h->model_id, d);
  if (d > 64 && !big) return fail(h, AMH_EINVAL, "amh_pooled_stats: d > 64 needs d % 32 == 0 in the pooled mode");
  if (h->model_id == AMH_MODEL_EXTERNAL)
    return fail(h, AMH_EINVAL, "amh_pooled_stats: the pooled mode needs a device potential (not external)");
  const int cpw = amh::pooled_cpw(num_chains);
  const int64_t chunk = (int64_t)amh::kPoolWaves * cpw;
  const int64_t n_chunks = big ? amh::pooled_big_chunks(num_chains, d) : (num_chains + chunk - 1) / chunk;
  const int64_t vrow = big ? amh::pooled_big_tile_V(d) : d + (int64_t)d * (d + 1) / 2 + 2;
  const size_t need = (size_t)amh::pooled_scratch_rows(n_chunks) * (size_t)vrow * sizeof(double);
  if (need > h->partials_bytes) {
    if (h->partials) {
      (void)hipStreamSynchronize((hipStream_t)stream);  // a queued launch may still use the old scratch
      (void)hipFree(h->partials);
    }
    h->partials = nullptr;
    h->partials_bytes = 0;
    e = hipMalloc(&h->partials, need);
    if (e != hipSuccess) return hip_fail(h, e, "amh_pooled_stats/hipMalloc");
    h->partials_bytes = need;
  }
  amh::PooledStatsParams p{};
  p.C = num_chains;
  p.d = d;
  p.i = in->i;
  p.z = in->z;
  p.pe = in->potential_energy;
  p.keys = in->rng_key;
  p.mu = in->loc;
  p.L = in->scale;
  p.lam = in->log_step_size;
  p.eps = h->cfg.eps;
  p.z_out = z_out;
  p.pe_out = pe_out;
  p.partials = h->partials;
  p.model = h->model;
  p.k_steps = k_steps;
  if (big) {
    // xprop + U(xprop) of the unfused path, or the fused path's A-operand copies
    const size_t nb = ((size_t)num_chains * (size_t)(d + 1) + (size_t)amh::pooled_big_pack_floats(d)) * sizeof(float);
    h->big_ready_C = -1;
    void* const split_was = h->split_buf;
    int rc = grow(h, &h->split_buf, &h->split_bytes, nb, stream, "amh_pooled_stats/hipMalloc");
    if (rc != AMH_OK) return rc;
    // the copies are current only when the previous update of this call wrote
    // them into this very buffer (amh_pooled_step_k; d > 64 fused path)
    p.pack_ready = (pack_ready && d != 64 && h->split_buf == split_was) ? 1 : 0;
    {
      // noise drawn ahead by the update launch (records checked per chain
      // by the stats kernel, so a stale or foreign buffer is never used)
      const size_t nn = (size_t)num_chains * (16 + (size_t)d * sizeof(float));
      if (nn > h->noise_bytes) {
        rc = grow(h, &h->noise_buf, &h->noise_bytes, nn, stream, "amh_pooled_stats/hipMalloc");
        if (rc != AMH_OK) return rc;
        h->noise_cap = num_chains;
        e = hipMemsetAsync(h->noise_buf, 0xFF, (size_t)num_chains * 16, (hipStream_t)stream);  // i = -1: no match
        if (e != hipSuccess) return hip_fail(h, e, "amh_pooled_stats/hipMemsetAsync");
      }
      p.xrec = (const uint4*)h->noise_buf;
      p.xi = h->noise_buf + 4 * h->noise_cap;
      p.xi_cap = h->noise_cap;
      h->noise_C = num_chains;
      h->noise_keys = in->rng_key;
      if (prep_for_update) {  // grown here: pooled_update_impl's grow is then a no-op
        const size_t un = ((size_t)d * (d + 4) / 2 + 8 + (size_t)d) * sizeof(float);
        const bool fresh = un > h->upd_bytes;
        rc = grow(h, &h->upd_buf, &h->upd_bytes, un, stream, "amh_pooled_stats/hipMalloc");
        if (rc != AMH_OK) return rc;
        if (fresh) {
          e = hipMemsetAsync(h->upd_buf, 0, h->upd_bytes, (hipStream_t)stream);
          if (e != hipSuccess) return hip_fail(h, e, "amh_pooled_stats/hipMemsetAsync");
        }
      }
    }
    // one launch sequence per step of the block, the sums accumulated; d = 64:
    // the block's K steps in one launch (pooled_fused64_kernel, p.k_steps)
    const int32_t n_launch = (d == 64) ? 1 : k_steps;
    for (int32_t t0 = 0; t0 < n_launch; ++t0) {
      const int32_t t = (d == 64) ? k_steps - 1 : t0;  // the step the launch ends with
      p.i_add = (d == 64) ? 0 : t;
      p.accumulate = (d == 64) ? 0 : t > 0;
      if (prep_for_update && d != 64 && t == k_steps - 1) {
        p.prep.cov = in->cov;
        p.prep.i = in->i;
        p.prep.scratch = h->upd_buf;
        p.prep.N = (double)num_chains * (double)k_steps;
        p.prep.W = h->cfg.num_warmup;
        p.prep.K = k_steps;
        p.prep.a = h->cfg.lr_decay;
        if (sigma_ready) *sigma_ready = true;
      }
      if (t0 > 0) {
        p.z = z_out;
        p.pe = pe_out;
      }
      p.defer_reduce = (prep_for_update && deferred && d == 64 && t == k_steps - 1 && !reduce_fusion_off()) ? 1 : 0;
      if (p.defer_reduce) {
        deferred->partials = (const float*)h->partials;
        deferred->n_chunks = n_chunks;
        deferred->accumulate = p.accumulate;
      }
      e = amh::run_pooled_big_stats(p, h->split_buf, h->split_buf + (size_t)num_chains * d, sums,
                                    (hipStream_t)stream);
      if (e != hipSuccess) return hip_fail(h, e, "amh_pooled_stats(MFMA path)");
      p.pack_ready = 1;  // the K steps of a pooled block share the frozen factor
    }
    return AMH_OK;
  }
  e = amh::run_pooled_stats(h->model_id, p, sums, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(h, e, "amh_pooled_stats");
  return AMH_OK;
}

static int pooled_update_impl(amh_handle* h, const double* sums, const amh_pooled_state* in,
                              const amh_pooled_state* out, int32_t k_steps, void* stream, bool sigma_ready,
                              const DeferredReduce* deferred = nullptr, float* pack_out = nullptr);

extern "C" {

int amh_pooled_stats_k(amh_handle* h, int64_t num_chains, const amh_pooled_state* in, int32_t k_steps,
                       float* z_out, float* pe_out, double* sums, void* stream) {
  return pooled_stats_impl(h, num_chains, in, k_steps, z_out, pe_out, sums, stream, false, nullptr);
}

int amh_pooled_stats(amh_handle* h, int64_t num_chains, const amh_pooled_state* in, float* z_out, float* pe_out,
                     double* sums, void* stream) {
  return amh_pooled_stats_k(h, num_chains, in, 1, z_out, pe_out, sums, stream);
}

int amh_pooled_update_k(amh_handle* h, const double* sums, const amh_pooled_state* in, const amh_pooled_state* out,
                        int32_t k_steps, void* stream) {
  return pooled_update_impl(h, sums, in, out, k_steps, stream, false);
}

}  // extern "C"

static int pooled_update_impl(amh_handle* h, const double* sums, const amh_pooled_state* in,
                              const amh_pooled_state* out, int32_t k_steps, void* stream, bool sigma_ready,
                              const DeferredReduce* deferred, float* pack_out) {
  if (!h) return fail(nullptr, AMH_EINVAL, "amh_pooled_update: null handle");
  if (!sums || !pooled_ok(in) || !pooled_ok(out)) return fail(h, AMH_EINVAL, "amh_pooled_update: bad arguments");
  if (k_steps < 1 || h->cfg.num_warmup % k_steps != 0)
    return fail(h, AMH_EINVAL, "amh_pooled_update: k_steps must be >= 1 and divide num_warmup");
  if (h->cfg.dim > 64 && !amh::pooled_big_model(h->model_id, h->cfg.dim))
    return fail(h, AMH_EINVAL, "amh_pooled_update: d > 64 needs d % 32 == 0 in the pooled mode");
  if (int rc = check_device_flag(h)) return rc;
  hipError_t e = hipSetDevice(h->device);
  if (e != hipSuccess) return hip_fail(h, e, "amh_pooled_update/hipSetDevice");
  amh::PooledUpdateParams p{};
  p.d = h->cfg.dim;
  p.W = h->cfg.num_warmup;
  p.a = h->cfg.lr_decay;
  p.target = h->cfg.target_accept_prob;
  p.sums = sums;
  p.in = *in;
  p.out = *out;
  p.K = k_steps;
  if (amh::pooled_big_model(h->model_id, p.d)) {
    const size_t need = ((size_t)p.d * (p.d + 4) / 2 + 8 + (size_t)p.d) * sizeof(float);
    const bool fresh = need > h->upd_bytes;
    int rc = grow(h, &h->upd_buf, &h->upd_bytes, need, stream, "amh_pooled_update/hipMalloc");
    if (rc != AMH_OK) return rc;
    if (fresh) {  // the post kernel's arrival ticket starts at zero (its last block resets it)
      e = hipMemsetAsync(h->upd_buf, 0, h->upd_bytes, (hipStream_t)stream);
      if (e != hipSuccess) return hip_fail(h, e, "amh_pooled_update/hipMemsetAsync");
    }
    p.scratch = h->upd_buf;
    if (p.d == 64 && h->err_host == nullptr) {
      e = hipHostMalloc((void**)&h->err_host, sizeof(int), hipHostMallocMapped);
      if (e == hipSuccess) {
        *h->err_host = 0;
        e = hipHostGetDevicePointer((void**)&h->err_dev, h->err_host, 0);
      }
      if (e != hipSuccess) return hip_fail(h, e, "amh_pooled_update/hipHostMalloc");
    }
    p.err_flag = h->err_dev;
    p.pack_out = (p.d > 64) ? pack_out : nullptr;
    if (h->noise_buf && h->noise_C > 0 && h->noise_C <= h->noise_cap && in->rng_key == h->noise_keys &&
        !noise_ahead_off()) {
      p.noise_C = h->noise_C;  // the chains (and keys) of the stats call this update follows
      p.keys = (const uint32_t*)in->rng_key;
      p.xrec = (uint4*)h->noise_buf;
      p.xi = h->noise_buf + 4 * h->noise_cap;
    }
    if (deferred && deferred->partials) {
      p.red_partials = deferred->partials;
      p.red_chunks = deferred->n_chunks;
      p.red_accumulate = deferred->accumulate;
      p.red_blocks = amh::pooled_reduce64_blocks(amh::pooled_big_tile_V(p.d));
      p.sums_out = const_cast<double*>(sums);
    }
    e = amh::run_pooled_big_update(p, (hipStream_t)stream, sigma_ready);
  } else {
    e = amh::run_pooled_update(p, (hipStream_t)stream);
  }
  if (e != hipSuccess) return hip_fail(h, e, "amh_pooled_update");
  return AMH_OK;
}

extern "C" {

int amh_pooled_update(amh_handle* h, const double* sums, const amh_pooled_state* in, const amh_pooled_state* out,
                      void* stream) {
  return amh_pooled_update_k(h, sums, in, out, 1, stream);
}

int amh_pooled_step_k(amh_handle* h, int64_t num_chains, const amh_pooled_state* in, const amh_pooled_state* out,
                      int32_t n_steps, int32_t sync_every, double* sums, void* stream) {
  if (n_steps < 0 || sync_every < 1 || n_steps % sync_every != 0)
    return fail(h, AMH_EINVAL, "amh_pooled_step: n_steps must be a non-negative multiple of sync_every");
  const amh_pooled_state* src = in;
  const bool big = h && h->model_id && amh::pooled_big_model(h->model_id, h->cfg.dim) && h->cfg.dim > 64;
  for (int32_t t = 0; t < n_steps; t += sync_every) {
    bool ready = false;  // one rank, no exchange: the reduction also forms Sigma'
    DeferredReduce dr;   // (d = 64: or is left to the update launch)
    // d > 64: from the second block on, the stats launch's A-operand copy of
    // the factor was written by the previous update's post kernel
    int rc = pooled_stats_impl(h, num_chains, src, sync_every, out->z, out->potential_energy, sums, stream, true,
                               &ready, &dr, t > 0);
    if (rc != AMH_OK) return rc;
    rc = pooled_update_impl(h, sums, src, out, sync_every, stream, ready, &dr,
                            (big && t + sync_every < n_steps) ? h->split_buf : nullptr);
    if (rc != AMH_OK) return rc;
    src = out;
  }
  return AMH_OK;
}

int amh_pooled_step(amh_handle* h, int64_t num_chains, const amh_pooled_state* in, const amh_pooled_state* out,
                    int32_t n_steps, double* sums, void* stream) {
  return amh_pooled_step_k(h, num_chains, in, out, n_steps, 1, sums, stream);
}

// ncclAllReduce / ncclGetErrorString of the RCCL instance already in the
// process (the caller created `comm` with it: torch's librccl.so.1, found by
// soname without loading anything), else the system librccl.so.1
typedef int (*nccl_allreduce_fn)(const void*, void*, size_t, int, int, void*, void*);
typedef const char* (*nccl_errstr_fn)(int);
static void* rccl_handle() {
  static void* hd = nullptr;
  if (hd == nullptr) {
    hd = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (hd == nullptr) hd = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (hd == nullptr) hd = dlopen("librccl.so.1", RTLD_NOW);
  }
  return hd;
}

int amh_pooled_allreduce(amh_handle* h, double* sums, int64_t n, void* rccl_comm, void* stream) {
  if (!h) return fail(nullptr, AMH_EINVAL, "amh_pooled_allreduce: null handle");
  if (!sums || !rccl_comm || n < 0) return fail(h, AMH_EINVAL, "amh_pooled_allreduce: null sums / communicator");
  void* hd = rccl_handle();
  auto ar = hd ? (nccl_allreduce_fn)dlsym(hd, "ncclAllReduce") : nullptr;
  if (ar == nullptr) return fail(h, AMH_EHIP, "amh_pooled_allreduce: librccl not found");
  constexpr int kNcclFloat64 = 8, kNcclSum = 0;
  const int rc = ar(sums, sums, (size_t)n, kNcclFloat64, kNcclSum, rccl_comm, stream);
  if (rc != 0) {
    auto es = (nccl_errstr_fn)dlsym(hd, "ncclGetErrorString");
    return fail(h, AMH_EHIP, std::string("amh_pooled_allreduce: ncclAllReduce: ") + (es ? es(rc) : "error") +
                                 " (ncclResult " + std::to_string(rc) + ")");
  }
  return AMH_OK;
}

#ifdef AMH_STAMPS
// diagnostic build only: copy the step kernel's per-wave phase stamps
int amh_diag_stamps(void* host, int64_t bytes) {
  return amh::diag_stamps_copy(host, (size_t)bytes) == hipSuccess ? 0 : -1;
}
// pooled large-d update kernel phase totals (8 x u64)
int amh_diag_upd_stamps(void* host) { return amh::diag_upd_stamps_copy(host) == hipSuccess ? 0 : -1; }
// pooled d = 64 fused stats kernel phase totals (16 x u64, block 0 thread 0)
int amh_diag_f64_stamps(void* host) { return amh::diag_f64_stamps_copy(host) == hipSuccess ? 0 : -1; }
// pooled d = 64 update launch timeline (16 x u64, 100 MHz clock; copied, then cleared)
int amh_diag_u64_timeline(void* host) { return amh::diag_u64_timeline_copy(host) == hipSuccess ? 0 : -1; }
#endif
}  // extern "C"
