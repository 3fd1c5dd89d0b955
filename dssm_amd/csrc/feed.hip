// Host data path of the DSSM step, native: the reference's text -> sparse
// feed pipeline and an asynchronous pinned-memory feeder for the device CSR.
//
// Reference pipeline (semantic_matching/dssm/new_dssm.py:26-49, utils/utils.py):
//   get_data_set_comment (utils.py:368-421): per TSV line prefix/title -> pre_process (:424-437:
//   strip, drop http(s) short links, keep only U+4E00..U+9FA5, 0-9, A-Z, a-z) -> one character per
//   token, space separated;
//   CountVectorizer(token_pattern=r"(?u)\b\w+\b") fit on doc + query + doc_neg, transform ->
//   scipy CSR of counts (new_dssm.py:37-45), TRIGRAM_D = vocabulary size;
//   pull_batch (utils.py:45-61): row slices [b*BS, (b+1)*BS) of query / doc and [b*BS*NEG, ...)
//   of doc_neg fed as three COO tensors.
//
// Here:
//   * dssm_text_clean: pre_process, byte-exact for UTF-8 input;
//   * dssm_vocab_*: the CountVectorizer for that alphabet (lowercase=True; a token is a maximal
//     run of word characters -- [0-9A-Za-z_] and U+4E00..U+9FA5, the only ones pre_process
//     keeps -- any other code point separates tokens); vocabulary ids in code-point order of the
//     token strings (sklearn sorts feature names), counts per document as CSR with sorted columns;
//   * dssm_feeder_*: the device path's combined CSR [q(BS); pos(BS); neg(BS*NEG)] of batch b
//     assembled by a host worker thread from the three CSR matrices into pinned slots and copied
//     to device slots on the feeder's own stream, so the H2D of batch b+1 overlaps step b; the
//     consumer's stream waits on the slot's event (no host sync on the step path).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/dssm.h"

namespace dssm {
int report_error(int code, const char* msg);  // plan.hip: sets dssm_last_error()
}

namespace {

int ferr(int code, const std::string& m) { return dssm::report_error(code, m.c_str()); }

// ---- UTF-8 ------------------------------------------------------------------------------------
// Decode one code point at s[i] (advancing i); invalid bytes decode as U+FFFD (one byte).
uint32_t next_cp(const std::string& s, size_t& i) {
  const unsigned char c = (unsigned char)s[i];
  int n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
  if (n == 0 || i + n > s.size()) {
    ++i;
    return 0xFFFD;
  }
  uint32_t cp = n == 1 ? c : n == 2 ? (c & 0x1F) : n == 3 ? (c & 0x0F) : (c & 0x07);
  for (int k = 1; k < n; ++k) {
    const unsigned char d = (unsigned char)s[i + k];
    if ((d >> 6) != 2) {
      ++i;
      return 0xFFFD;
    }
    cp = (cp << 6) | (d & 0x3F);
  }
  i += n;
  return cp;
}

bool keep_cp(uint32_t cp) {  // pre_process's final character class (utils.py:436)
  return (cp >= 0x4E00 && cp <= 0x9FA5) || (cp >= '0' && cp <= '9') || (cp >= 'A' && cp <= 'Z') ||
         (cp >= 'a' && cp <= 'z');
}

bool url_cp(unsigned char c) {  // (?:[a-zA-Z]|[0-9]|[$-_@.&+]|[!*\(\),]|%XX)  ('%' is in $-_)
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') ||
         (c >= '$' && c <= '_') || c == '@' || c == '.' || c == '&' || c == '+' || c == '!' ||
         c == '*' || c == '(' || c == ')' || c == ',';
}

// re.findall(r'http[s]?://(...)+', line): leftmost, non-overlapping, greedy
std::vector<std::string> find_urls(const std::string& s) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i < s.size()) {
    if (s.compare(i, 4, "http") == 0) {
      size_t j = i + 4;
      if (j < s.size() && s[j] == 's' && s.compare(j + 1, 3, "://") == 0) j += 4;
      else if (s.compare(j, 3, "://") == 0) j += 3;
      else {
        ++i;
        continue;
      }
      size_t k = j;
      while (k < s.size() && url_cp((unsigned char)s[k])) ++k;
      if (k > j) {
        out.push_back(s.substr(i, k - i));
        i = k;
        continue;
      }
    }
    ++i;
  }
  return out;
}

void replace_all(std::string& s, const std::string& from) {
  if (from.empty()) return;
  std::string r;
  r.reserve(s.size());
  size_t i = 0;
  for (size_t p; (p = s.find(from, i)) != std::string::npos; i = p + from.size()) r.append(s, i, p - i);
  r.append(s, i, std::string::npos);
  s.swap(r);
}

// pre_process (utils.py:424-437).  strip() only trims whitespace, which the final filter drops
// anyway and which no URL contains, so it does not change the result.
std::string clean(const std::string& line) {
  std::string s = line;
  for (const std::string& u : find_urls(line)) replace_all(s, u);  // line.replace(url, "") per url
  std::string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size();) {
    const size_t b = i;
    const uint32_t cp = next_cp(s, i);
    if (keep_cp(cp)) out.append(s, b, i - b);
  }
  return out;
}

bool word_cp(uint32_t cp) { return keep_cp(cp) || cp == '_'; }

// CountVectorizer's analyzer for this alphabet: lowercase, then maximal runs of word characters
template <typename F>
void tokens(const char* text, F&& f) {
  const std::string s(text);
  std::string tok;
  for (size_t i = 0; i < s.size();) {
    const size_t b = i;
    const uint32_t cp = next_cp(s, i);
    if (word_cp(cp)) {
      if (cp >= 'A' && cp <= 'Z') tok.push_back((char)(cp + 32));
      else tok.append(s, b, i - b);
    } else if (!tok.empty()) {
      f(tok);
      tok.clear();
    }
  }
  if (!tok.empty()) f(tok);
}

}  // namespace

struct dssm_vocab {
  std::unordered_map<std::string, int32_t> id;  // -1 until finalised
  std::vector<std::string> names;               // sorted feature names after finalise
  bool final_ = false;
};

struct dssm_feeder {
  // host CSR matrices (caller-owned, must outlive the feeder)
  const int64_t* ip[3];
  const int32_t* ix[3];
  const float* val[3];
  int64_t nrows[3];
  int bs, neg, nslots;
  int64_t max_nnz;
  hipStream_t stream = nullptr;
  struct Slot {
    int32_t* h_ip = nullptr;  // pinned
    int32_t* h_ix = nullptr;
    float* h_val = nullptr;
    int32_t* d_ip = nullptr;  // device
    int32_t* d_ix = nullptr;
    float* d_val = nullptr;
    hipEvent_t done = nullptr;      // this slot's copy completed (feeder stream)
    hipEvent_t consumed = nullptr;  // the consumer's last reader of the slot (its stream)
    bool consumed_set = false;
    int64_t batch = -1;
    int64_t nnz = 0;
    bool ready = false;  // copy enqueued
    int err = 0;
  };
  std::vector<Slot> slots;
  std::thread worker;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<int, int64_t>> queue;  // (slot, batch)
  bool stop = false;
};

namespace {

// Combined CSR [q(BS); pos(BS); neg(BS*NEG)] of batch b into the slot's pinned buffers
int assemble(dssm_feeder* F, dssm_feeder::Slot& s, int64_t b) {
  const int64_t r0[3] = {b * F->bs, b * F->bs, b * F->bs * F->neg};
  const int64_t nr[3] = {F->bs, F->bs, (int64_t)F->bs * F->neg};
  int64_t nnz = 0, row = 0;
  s.h_ip[0] = 0;
  for (int m = 0; m < 3; ++m) {
    if (r0[m] + nr[m] > F->nrows[m]) return DSSM_E_INVALID;
    const int64_t e0 = F->ip[m][r0[m]], e1 = F->ip[m][r0[m] + nr[m]];
    if (nnz + (e1 - e0) > F->max_nnz) return DSSM_E_INVALID;
    std::memcpy(s.h_ix + nnz, F->ix[m] + e0, sizeof(int32_t) * (e1 - e0));
    std::memcpy(s.h_val + nnz, F->val[m] + e0, sizeof(float) * (e1 - e0));
    for (int64_t r = 0; r < nr[m]; ++r)
      s.h_ip[row + r + 1] = (int32_t)(nnz + F->ip[m][r0[m] + r + 1] - e0);
    row += nr[m];
    nnz += e1 - e0;
  }
  s.nnz = nnz;
  return DSSM_OK;
}

void worker_loop(dssm_feeder* F) {
  for (;;) {
    std::pair<int, int64_t> job;
    {
      std::unique_lock<std::mutex> lk(F->mu);
      F->cv.wait(lk, [&] { return F->stop || !F->queue.empty(); });
      if (F->stop && F->queue.empty()) return;
      job = F->queue.front();
      F->queue.pop_front();
    }
    dssm_feeder::Slot& s = F->slots[job.first];
    // the slot's previous copy must have left the pinned buffers before they are rewritten
    hipEventSynchronize(s.done);
    int rc = assemble(F, s, job.second);
    const int64_t rows = (int64_t)F->bs * (2 + F->neg);
    if (rc == DSSM_OK) {
      // device slot reuse: the copy waits (on the device) for the consumer's release
      hipError_t e = s.consumed_set ? hipStreamWaitEvent(F->stream, s.consumed, 0) : hipSuccess;
      if (e == hipSuccess)
        e = hipMemcpyAsync(s.d_ip, s.h_ip, sizeof(int32_t) * (rows + 1), hipMemcpyHostToDevice, F->stream);
      if (e == hipSuccess && s.nnz)
        e = hipMemcpyAsync(s.d_ix, s.h_ix, sizeof(int32_t) * s.nnz, hipMemcpyHostToDevice, F->stream);
      if (e == hipSuccess && s.nnz)
        e = hipMemcpyAsync(s.d_val, s.h_val, sizeof(float) * s.nnz, hipMemcpyHostToDevice, F->stream);
      if (e == hipSuccess) e = hipEventRecord(s.done, F->stream);
      if (e != hipSuccess) rc = DSSM_E_HIP;
    }
    {
      std::lock_guard<std::mutex> lk(F->mu);
      s.err = rc;
      s.batch = job.second;
      s.ready = true;
    }
    F->cv.notify_all();
  }
}

}  // namespace

extern "C" {

int dssm_text_clean(const char* text, char* out, size_t cap, size_t* len) {
  if (!text || !len) return ferr(DSSM_E_INVALID, "null argument");
  const std::string r = clean(text);
  *len = r.size();
  if (out && cap) {
    const size_t n = std::min(cap - 1, r.size());
    std::memcpy(out, r.data(), n);
    out[n] = 0;
  }
  return DSSM_OK;
}

int dssm_vocab_create(dssm_vocab** out) {
  if (!out) return ferr(DSSM_E_INVALID, "null argument");
  *out = new dssm_vocab();
  return DSSM_OK;
}

int dssm_vocab_destroy(dssm_vocab* v) {
  delete v;
  return DSSM_OK;
}

int dssm_vocab_fit(dssm_vocab* v, const char* const* texts, int64_t n) {
  if (!v || (n && !texts)) return ferr(DSSM_E_INVALID, "null argument");
  if (v->final_) return ferr(DSSM_E_INVALID, "vocabulary already finalised");
  for (int64_t i = 0; i < n; ++i)
    tokens(texts[i], [&](const std::string& t) { v->id.emplace(t, -1); });
  return DSSM_OK;
}

int64_t dssm_vocab_finalize(dssm_vocab* v) {
  if (!v) return ferr(DSSM_E_INVALID, "null argument");
  v->names.clear();
  for (auto& kv : v->id) v->names.push_back(kv.first);
  std::sort(v->names.begin(), v->names.end());  // UTF-8 byte order == code-point order
  for (size_t i = 0; i < v->names.size(); ++i) v->id[v->names[i]] = (int32_t)i;
  v->final_ = true;
  return (int64_t)v->names.size();
}

int64_t dssm_vocab_size(const dssm_vocab* v) { return v ? (int64_t)v->names.size() : -1; }

int dssm_vocab_name(const dssm_vocab* v, int64_t i, char* out, size_t cap) {
  if (!v || i < 0 || i >= (int64_t)v->names.size() || !out || !cap)
    return ferr(DSSM_E_INVALID, "bad argument");
  const std::string& s = v->names[i];
  const size_t n = std::min(cap - 1, s.size());
  std::memcpy(out, s.data(), n);
  out[n] = 0;
  return (int)s.size();
}

int dssm_vocab_add(dssm_vocab* v, const char* name) {  // restore a saved vocabulary, in id order
  if (!v || !name) return ferr(DSSM_E_INVALID, "null argument");
  v->id[name] = (int32_t)v->names.size();
  v->names.emplace_back(name);
  v->final_ = true;
  return DSSM_OK;
}

// CRC-32C (reflected polynomial 0x82F63B78) extending a finished CRC, as leveldb / TF's
// crc32c::Extend: the TF checkpoint writer / reader (dssm_amd/tfckpt.py) checks every tensor with it.
__attribute__((target("sse4.2"))) uint32_t dssm_crc32c(uint32_t crc, const void* data, size_t n) {
  const unsigned char* p = static_cast<const unsigned char*>(data);
  uint64_t l = ~crc;
  for (; n && (reinterpret_cast<uintptr_t>(p) & 7); --n) l = __builtin_ia32_crc32qi((uint32_t)l, *p++);
  for (; n >= 8; n -= 8, p += 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    l = __builtin_ia32_crc32di(l, w);
  }
  for (; n; --n) l = __builtin_ia32_crc32qi((uint32_t)l, *p++);
  return ~(uint32_t)l;
}

// Counts per document (CSR, sorted columns; unknown tokens dropped like sklearn's transform).
// Pass indices/values NULL to size: *nnz_out = total non-zeros (indptr filled either way).
int dssm_vocab_transform(const dssm_vocab* v, const char* const* texts, int64_t n, int64_t* indptr,
                         int32_t* indices, float* values, int64_t cap, int64_t* nnz_out) {
  if (!v || !indptr || !nnz_out || (n && !texts)) return ferr(DSSM_E_INVALID, "null argument");
  if (!v->final_) return ferr(DSSM_E_INVALID, "vocabulary not finalised");
  std::vector<int32_t> ids;
  int64_t nnz = 0;
  indptr[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    ids.clear();
    tokens(texts[i], [&](const std::string& t) {
      auto it = v->id.find(t);
      if (it != v->id.end()) ids.push_back(it->second);
    });
    std::sort(ids.begin(), ids.end());
    for (size_t k = 0; k < ids.size();) {
      size_t e = k;
      while (e < ids.size() && ids[e] == ids[k]) ++e;
      if (indices) {
        if (nnz >= cap) return ferr(DSSM_E_INVALID, "transform: capacity exceeded");
        indices[nnz] = ids[k];
        values[nnz] = (float)(e - k);
      }
      ++nnz;
      k = e;
    }
    indptr[i + 1] = nnz;
  }
  *nnz_out = nnz;
  return DSSM_OK;
}

int dssm_feeder_create(const int64_t* const* indptr, const int32_t* const* indices,
                       const float* const* values, const int64_t* rows, int query_bs, int neg,
                       int64_t max_nnz, int nslots, dssm_feeder** out) {
  if (!indptr || !indices || !values || !rows || !out || query_bs < 1 || neg < 1 || nslots < 2 ||
      max_nnz < 0)
    return ferr(DSSM_E_INVALID, "bad feeder argument");
  auto* F = new dssm_feeder();
  for (int m = 0; m < 3; ++m) {
    F->ip[m] = indptr[m];
    F->ix[m] = indices[m];
    F->val[m] = values[m];
    F->nrows[m] = rows[m];
  }
  F->bs = query_bs;
  F->neg = neg;
  F->nslots = nslots;
  F->max_nnz = max_nnz;
  const int64_t R = (int64_t)query_bs * (2 + neg);
  F->slots.resize(nslots);
  bool ok = hipStreamCreateWithFlags(&F->stream, hipStreamNonBlocking) == hipSuccess;
  const size_t cap = (size_t)std::max<int64_t>(max_nnz, 1);
  for (auto& s : F->slots) {
    ok = ok && hipHostMalloc((void**)&s.h_ip, sizeof(int32_t) * (R + 1), hipHostMallocDefault) == hipSuccess;
    ok = ok && hipHostMalloc((void**)&s.h_ix, sizeof(int32_t) * cap, hipHostMallocDefault) == hipSuccess;
    ok = ok && hipHostMalloc((void**)&s.h_val, sizeof(float) * cap, hipHostMallocDefault) == hipSuccess;
    ok = ok && hipMalloc((void**)&s.d_ip, sizeof(int32_t) * (R + 1)) == hipSuccess;
    ok = ok && hipMalloc((void**)&s.d_ix, sizeof(int32_t) * cap) == hipSuccess;
    ok = ok && hipMalloc((void**)&s.d_val, sizeof(float) * cap) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&s.done, hipEventDisableTiming) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&s.consumed, hipEventDisableTiming) == hipSuccess;
  }
  if (!ok) {
    dssm_feeder_destroy(F);
    return ferr(DSSM_E_HIP, "feeder: pinned / device slot allocation failed");
  }
  F->worker = std::thread(worker_loop, F);
  *out = F;
  return DSSM_OK;
}

int dssm_feeder_submit(dssm_feeder* F, int slot, int64_t batch) {
  if (!F || slot < 0 || slot >= F->nslots || batch < 0) return ferr(DSSM_E_INVALID, "bad argument");
  {
    std::lock_guard<std::mutex> lk(F->mu);
    for (const auto& q : F->queue)
      if (q.first == slot) return ferr(DSSM_E_INVALID, "slot already queued");
    F->slots[slot].ready = false;
    F->queue.emplace_back(slot, batch);
  }
  F->cv.notify_all();
  return DSSM_OK;
}

// Wait (host) until the slot's copy is ENQUEUED, make `stream` wait (device) for its completion,
// and hand out the device CSR pointers.
int dssm_feeder_acquire(dssm_feeder* F, int slot, void* stream, const int32_t** indptr,
                        const int32_t** indices, const float** values, int64_t* nnz) {
  if (!F || slot < 0 || slot >= F->nslots) return ferr(DSSM_E_INVALID, "bad argument");
  dssm_feeder::Slot& s = F->slots[slot];
  {
    std::unique_lock<std::mutex> lk(F->mu);
    F->cv.wait(lk, [&] { return s.ready; });
  }
  if (s.err) return ferr(s.err, "feeder: batch assembly failed (rows or max_nnz out of range)");
  if (hipStreamWaitEvent((hipStream_t)stream, s.done, 0) != hipSuccess)
    return ferr(DSSM_E_HIP, "feeder: hipStreamWaitEvent");
  if (indptr) *indptr = s.d_ip;
  if (indices) *indices = s.d_ix;
  if (values) *values = s.d_val;
  if (nnz) *nnz = s.nnz;
  return DSSM_OK;
}

// After the step reading the slot is enqueued on `stream`: the slot's next copy will wait (on the
// device) for that work, so the slot can be resubmitted at once.
int dssm_feeder_release(dssm_feeder* F, int slot, void* stream) {
  if (!F || slot < 0 || slot >= F->nslots) return ferr(DSSM_E_INVALID, "bad argument");
  std::lock_guard<std::mutex> lk(F->mu);
  dssm_feeder::Slot& s = F->slots[slot];
  if (hipEventRecord(s.consumed, (hipStream_t)stream) != hipSuccess)
    return ferr(DSSM_E_HIP, "feeder: hipEventRecord");
  s.consumed_set = true;
  return DSSM_OK;
}

int dssm_feeder_destroy(dssm_feeder* F) {
  if (!F) return DSSM_OK;
  if (F->worker.joinable()) {
    {
      std::lock_guard<std::mutex> lk(F->mu);
      F->stop = true;
    }
    F->cv.notify_all();
    F->worker.join();
  }
  if (F->stream) hipStreamSynchronize(F->stream);
  for (auto& s : F->slots) {
    if (s.h_ip) hipHostFree(s.h_ip);
    if (s.h_ix) hipHostFree(s.h_ix);
    if (s.h_val) hipHostFree(s.h_val);
    if (s.d_ip) hipFree(s.d_ip);
    if (s.d_ix) hipFree(s.d_ix);
    if (s.d_val) hipFree(s.d_val);
    if (s.done) hipEventDestroy(s.done);
    if (s.consumed) hipEventDestroy(s.consumed);
  }
  if (F->stream) hipStreamDestroy(F->stream);
  delete F;
  return DSSM_OK;
}

}  // extern "C"
