// a5x_host.cpp -- host side of liba5x: the C ABI declared in include/a5x.h.
//
//   * substitution tables: Go-exact parser (readSubstitutionTable, main.go:108-144;
//     decodeHexNotation, main.go:147-162) and the -t merge (main.go:40-50), then
//     compiled into the flat LDS-resident device table of a5x_format.h;
//   * dictionary splitting with bufio.ScanLines semantics (main.go:72-74);
//   * the per-batch device pipeline (keyspace -> scans -> plan -> expand) on one
//     HIP stream, replacing the goroutine-per-word dispatch and the single
//     channel writer of main.go:58-98;
//   * host-buffer convenience calls (a5x_keyspace, a5x_expand) that stage words
//     into HBM and stream the expanded bytes back to a sink.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <unordered_map>
#include <memory>
#include <vector>

#include "a5x.h"
#include "a5x_format.h"
#include "a5x_plan.h"
#include "a5x_gosem.h"
#include "a5x_launch.h"
#include "a5x_md.h"

namespace {

// ---------------------------------------------------------------------------
// the merged map[string][]string (keys in first-appearance order)
// ---------------------------------------------------------------------------
struct Table {
  std::vector<std::string> keys;
  std::vector<std::vector<std::string>> vals;
  std::unordered_map<std::string, uint32_t> index;

  void add(const std::string& k, const std::string& v) {
    auto it = index.find(k);
    uint32_t i;
    if (it == index.end()) {
      i = (uint32_t)keys.size();
      index.emplace(k, i);
      keys.push_back(k);
      vals.emplace_back();
    } else {
      i = it->second;
    }
    vals[i].push_back(v);
  }
  void clear() { keys.clear(); vals.clear(); index.clear(); }
  size_t nvals() const {
    size_t n = 0;
    for (auto& v : vals) n += v.size();
    return n;
  }
};

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;  // elements
};

}  // namespace

struct a5x_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  std::string devname;
  int cus = 0;

  Table table;
  bool table_dirty = true;
  std::vector<uint8_t> blob;
  uint8_t* d_table = nullptr;
  size_t d_table_cap = 0;
  uint32_t table_bytes = 0;
  // -r / -s / -s -r engines (a5x_modes.hip): sorted mode table + per-item state
  bool mtable_dirty = true;
  std::vector<uint8_t> mblob;
  uint8_t* d_mtab = nullptr;
  size_t d_mtab_cap = 0;
  uint32_t mtab_bytes = 0;
  DevBuf<uint64_t> m_nseg, m_seg_off, m_seg_bytes, m_seg_boff, m_tmp;
  DevBuf<uint8_t> m_item_fl;  // per item: the layout that expands it (a5x_modes.hip m_item)
  DevBuf<uint32_t> m_item_w;
  uint64_t m_items = 0;
  uint64_t m_nglob = 0;       // mode pass G words of the current batch (their list: glob)
  // hybrid fused digest: the non-FAST words of a batch gathered into a sub-batch
  DevBuf<uint32_t> hy_list;
  DevBuf<uint64_t> hy_lens, hy_off;
  DevBuf<uint8_t> hy_words;
  uint8_t* mgscr = nullptr;   // mode pass G scratch: A5X_G_SLOTS x a5x_mode_gslot_bytes(), on first use
  uint64_t mseg = 4096;  // candidates per mode-engine item (C5 -r: most words one item, sized by k_mode_count)
  uint64_t rov_need = 0;  // -r/-s FAST probe: overflow slots a previous batch needed (k_keyspace_rprobe)
  uint64_t cplx_need = 0;  // default mode: complex-word record slots a previous batch needed
  // -s / -s -r virtual words (k_keyspace_vsub, k_vwords_fill): the words left to the mode
  // engine, per-word sub-word counts / record sizes and their scans, the sub-word records,
  // and the virtual word list k_expand_fast runs on
  DevBuf<uint32_t> m_vl;
  DevBuf<uint64_t> vn, vrsz, vpre, vrpre, vrec, vrec2, vcand_off, vbyte_off;
  DevBuf<uint16_t> vocc;  // per word 16 u16: occurrence rows (k_keyspace_thread -> k_keyspace_vsub)
  DevBuf<uint32_t> vflags, vroff, vmap, vobase;
  uint64_t vrec_need = 0;  // sub-word record u64 a previous batch needed
  // fused digest + lookup (a5x_digest.hip)
  int t_algo = -1;
  uint64_t n_targets = 0;
  uint32_t t_bm_log2 = 0, t_has_zero = 0;
  uint64_t t_tmask = 0;
  DevBuf<uint32_t> t_bitmap;
  DevBuf<uint4> t_table;
  DevBuf<uint8_t> dg_scratch;
  DevBuf<uint64_t> dg_blk_cnt, dg_blk_pre, dg_cand_off, dg_byte_off;
  DevBuf<A5xHitRaw> dg_hits;
  hipEvent_t dev_ev[2] = {nullptr, nullptr};

  DevBuf<uint64_t> count, bytes, cand_off, byte_off, scan_tmp, locate;
  DevBuf<uint32_t> flags, defer, chunk_w0, slow_list, big_list, roff, cplx;
  DevBuf<uint64_t> segs;  // slow / BIG segment items
  DevBuf<uint32_t> glob;  // pass G word list (words beyond the pass-B LDS budget)
  DevBuf<uint32_t> m_cl, m_cl2;  // mode-engine word lists (FAST probe -> k_mode_count_thread -> k_mode_count)
  uint8_t* gscr = nullptr;  // pass G scratch: A5X_G_SLOTS x a5x_gslot_bytes(), allocated on first use
  DevBuf<uint64_t> rec;  // FAST plan records (keyspace tiles of FW_TILE_REC u64)
  uint32_t* d_scalars = nullptr;  // [0] defer_n, [1] nbig, [2] err, [3] nslow, [4] cplx_n, [5] slow segs, [6] BIG segs, [16..31] guard record
  uint32_t* h_scalars = nullptr;  // pinned
  uint64_t* h_totals = nullptr;   // pinned [0] cands [1] bytes [2..3] locate

  // host-API staging: words, and the double-buffered output stream of a5x_expand
  // (two HBM range buffers, two pinned host buffers, a copy stream; main.go:58-68)
  DevBuf<uint8_t> s_words, s_out[2];
  DevBuf<uint64_t> s_woff;
  uint8_t* h_out[2] = {nullptr, nullptr};
  size_t h_out_cap = 0;
  hipStream_t cstream = nullptr;
  hipEvent_t ev_exp[2] = {nullptr, nullptr}, ev_cpy[2] = {nullptr, nullptr};
  DevBuf<uint64_t> loc_q, loc_r;  // range-boundary queries / results (job_locate)

  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  // side stream: the per-word kernels (k_expand_slow / k_expand_b) of a range run beside
  // k_expand_fast (disjoint output bytes), joined back before the range completes
  hipStream_t sstream = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  uint64_t seg = 512;         // candidates per per-word-path segment (a radix round there costs ~64x a FAST one;
                              // C3 A/B: 512 / 256 -1 %, 4096 +8 %, 16384 +44 % -- the slow words run beside k_expand_fast)
  uint64_t chunk = 16384;     // candidates per expand wave (round-5 A/B, profiles/r05c_ab_chunk_16k.txt:
                              // C3 expansion 8.49-8.53 vs 8.62-8.76 ms at 8192, 8.56 at 32768)
  uint32_t waves_per_block = 4;
  uint32_t waves_per_block_fast = 1;
};

namespace {

int fail(a5x_ctx* c, int code, const char* fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    c->err = buf;
  }
  return code;
}

#define HIPCHK(c, x)                                                                              \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) return fail((c), A5X_E_HIP, "%s failed: %s", #x, hipGetErrorString(e_)); \
  } while (0)

template <typename T>
int grow(a5x_ctx* c, DevBuf<T>& b, size_t n) {
  if (n <= b.cap) return A5X_OK;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t want = n + n / 8 + 64;
  hipError_t e = hipMalloc((void**)&b.p, want * sizeof(T));
  if (e != hipSuccess) {
    b.p = nullptr;
    return fail(c, A5X_E_NOMEM, "hipMalloc(%zu bytes) failed: %s", want * sizeof(T), hipGetErrorString(e));
  }
  b.cap = want;
  return A5X_OK;
}

template <typename T>
void release(DevBuf<T>& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
}

// readSubstitutionTable on one file's bytes, merged into t (main.go:108-144 + 40-50)
int parse_table_into(a5x_ctx* c, Table& t, const uint8_t* d, size_t n) {
  using namespace a5x::gosem;
  Table ft;  // the file's own map, then appended per key like main.go:47-49
  size_t pos = 0;
  const uint8_t* line;
  size_t len;
  int r;
  while ((r = scan_line(d, n, &pos, &line, &len)) == 1) {
    const uint8_t* s = line;
    size_t m = len;
    trim_space(&s, &m);
    if (m == 0 || s[0] == '#') continue;
    const uint8_t* eq = (const uint8_t*)memchr(s, '=', m);
    if (!eq) continue;
    std::string k, v;
    const size_t kn = (size_t)(eq - s);
    if (!decode_hex_notation(s, kn, &k)) {
      fprintf(stderr, "Error decoding hex notation in key: %.*s\n", (int)m, (const char*)s);
      continue;
    }
    if (!decode_hex_notation(eq + 1, m - kn - 1, &v)) {
      fprintf(stderr, "Error decoding hex notation in value: %.*s\n", (int)m, (const char*)s);
      continue;
    }
    ft.add(k, v);
  }
  if (r < 0) return fail(c, A5X_E_TOOLONG, "bufio.Scanner: token too long");
  for (size_t i = 0; i < ft.keys.size(); i++)
    for (auto& v : ft.vals[i]) t.add(ft.keys[i], v);
  return A5X_OK;
}

// Compile the map into the device table blob of a5x_format.h.
// Static per-key facts of the -s / -s -r positional engines (k_mode_count_thread, the
// -s / -s -r FAST probe of k_keyspace_thread): bit 0 / 1 = the key passes m_pos_setup's
// positional checks in -s / -s -r for ANY word (one codepoint, ASCII if one byte; <= 14
// values (-s) or subs[0] (-s -r) of <= 15 valid UTF-8 bytes containing no key at all -- a
// superset of "no later pattern"); bits 8-19 / 20-31 = sum over those values of
// (len - klen) + 2048.
uint32_t key_pos_facts(const Table& t, const std::string& k, const std::vector<std::string>& vs) {
  if (t.keys.size() > 1024) return 0;  // (the containment test is O(keys^2))
  auto valid_utf8 = [](const std::string& v) {
    for (size_t i = 0; i < v.size();) {
      int sz = 0;
      const int r = a5x::gosem::decode_rune((const uint8_t*)v.data() + i, v.size() - i, &sz);
      if (r == a5x::gosem::kRuneError && sz == 1) return false;
      i += (size_t)sz;
    }
    return true;
  };
  auto has_key = [&](const std::string& v) {
    for (const std::string& kj : t.keys)
      if (!kj.empty() && v.find(kj) != std::string::npos) return true;
    return false;
  };
  int sz = 0;
  const int r0 = k.empty() ? 0 : a5x::gosem::decode_rune((const uint8_t*)k.data(), k.size(), &sz);
  const bool cp = k.size() >= 1 && k.size() <= 4 && sz == (int)k.size() && !(r0 == a5x::gosem::kRuneError && sz == 1) &&
                  !(sz == 1 && (uint8_t)k[0] >= 0x80);
  auto vok = [&](const std::string& v) { return v.size() <= 15 && valid_utf8(v) && !has_key(v); };
  bool ok2 = cp && vs.size() <= 14, ok3 = cp;
  int d2 = 0, d3 = 0;
  for (size_t v = 0; v < vs.size(); v++) {
    const bool o = vok(vs[v]);
    ok2 = ok2 && o;
    if (v == 0) { ok3 = ok3 && o; d3 = (int)vs[0].size() - (int)k.size(); }
    d2 += (int)vs[v].size() - (int)k.size();
  }
  return (ok2 ? 1u : 0u) | (ok3 ? 2u : 0u) | ((uint32_t)(d2 + 2048) & 0xFFFu) << 8 | ((uint32_t)(d3 + 2048) & 0xFFFu) << 20;
}

int compile_table(a5x_ctx* c) {
  const Table& t = c->table;
  std::vector<uint32_t> order;
  for (uint32_t i = 0; i < t.keys.size(); i++)
    if (!t.keys[i].empty()) order.push_back(i);
  // bucket by first byte, longest key first inside a bucket
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    const uint8_t fa = (uint8_t)t.keys[a][0], fb = (uint8_t)t.keys[b][0];
    if (fa != fb) return fa < fb;
    return t.keys[a].size() > t.keys[b].size();
  });
  if (order.size() > 65535) return fail(c, A5X_E_UNSUPPORTED, "table has %zu keys (max 65535)", order.size());
  std::vector<uint16_t> bucket(257, 0);
  for (uint32_t i : order) bucket[(uint8_t)t.keys[i][0] + 1]++;
  for (int b = 0; b < 256; b++) bucket[b + 1] += bucket[b];

  std::vector<A5xKey> keys;
  std::vector<A5xChoice> ch;
  std::vector<uint8_t> blob;
  uint32_t max_klen = 0, max_vlen = 0;
  auto add_choice = [&](const std::string& s) -> int {
    A5xChoice x;
    memset(&x, 0, sizeof x);
    if (s.size() > 65535) return -1;
    x.len = (uint16_t)s.size();
    for (size_t i = 0; i < s.size() && i < 4; i++) x.first4 |= (uint32_t)(uint8_t)s[i] << (8 * i);
    if (blob.size() + s.size() > 65535) return -1;
    x.blob_off = (uint16_t)blob.size();
    blob.insert(blob.end(), s.begin(), s.end());
    ch.push_back(x);
    return 0;
  };
  for (uint32_t i : order) {
    const std::string& k = t.keys[i];
    const auto& vs = t.vals[i];
    if (k.size() > 65535 || vs.size() > 65535)
      return fail(c, A5X_E_UNSUPPORTED, "table key/value list too large for the device table");
    A5xKey key;
    memset(&key, 0, sizeof key);
    key.pad0 = (uint16_t)(key_pos_facts(t, k, vs) & 3u);  // -s / -s -r FAST probe (r_unit)
    key.klen = (uint16_t)k.size();
    key.nvals = (uint16_t)vs.size();
    key.choice_base = (uint32_t)ch.size();
    int maxd = -65536;
    if (add_choice(k)) return fail(c, A5X_E_UNSUPPORTED, "device table blob exceeds 64 KiB");
    for (auto& v : vs) {
      if (add_choice(v)) return fail(c, A5X_E_UNSUPPORTED, "device table blob exceeds 64 KiB");
      key.sumlen += (uint32_t)v.size();
      maxd = std::max(maxd, (int)v.size() - (int)k.size());
      max_vlen = std::max(max_vlen, (uint32_t)v.size());
    }
    key.maxdelta = (int16_t)std::max(-32768, std::min(32767, maxd));
    {
      size_t mc = k.size();
      for (auto& v : vs) mc = std::max(mc, v.size());
      key.maxclen = (uint16_t)std::min<size_t>(mc, 65535);
    }
    for (auto& v : vs) {
      const long d = (long)v.size() - (long)k.size();
      if (d > 0) key.sum_dpos += (uint32_t)d; else key.sum_dneg += (uint32_t)(-d);
    }
    {
      size_t mn = k.size();
      for (auto& v : vs) mn = std::min(mn, v.size());
      key.minclen = (uint16_t)std::min<size_t>(mn, 65535);
    }
    max_klen = std::max(max_klen, (uint32_t)k.size());
    keys.push_back(key);
  }
  auto al16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  A5xTableHdr h;
  memset(&h, 0, sizeof h);
  h.magic = A5X_TABLE_MAGIC;
  h.nkeys = (uint32_t)keys.size();
  h.nchoices = (uint32_t)ch.size();
  h.off_bucket = sizeof(A5xTableHdr);
  h.off_keys = (uint32_t)al16(h.off_bucket + 257 * sizeof(uint16_t));
  h.off_choices = (uint32_t)al16(h.off_keys + keys.size() * sizeof(A5xKey));
  h.off_kmatch = (uint32_t)al16(h.off_choices + ch.size() * sizeof(A5xChoice));
  h.off_bucket2 = (uint32_t)al16(h.off_kmatch + std::max<size_t>(keys.size(), 1) * 8);
  h.off_cval = (uint32_t)al16(h.off_bucket2 + 256 * 4);
  h.off_blob = (uint32_t)al16(h.off_cval + std::max<size_t>(ch.size(), 1) * 8);
  h.blob_bytes = (uint32_t)blob.size();
  h.total_bytes = (uint32_t)al16(h.off_blob + blob.size() + 8);  // 8 B tail for 4-byte reads
  h.max_klen = max_klen;
  h.max_vlen = max_vlen;
  h.has_empty_key = t.index.count(std::string()) ? 1u : 0u;
  for (int b = 0; b < 256; b++) h.max_bucket = std::max<uint32_t>(h.max_bucket, bucket[b + 1] - bucket[b]);
  h.lead_only = 1;
  for (int b = 0x80; b < 0xC0; b++) h.lead_only = bucket[b + 1] > bucket[b] ? 0u : h.lead_only;
  if (h.total_bytes > A5X_TABLE_LDS_MAX)
    return fail(c, A5X_E_UNSUPPORTED, "device table is %u bytes (LDS staging max %u)", h.total_bytes,
                (unsigned)A5X_TABLE_LDS_MAX);
  c->blob.assign(h.total_bytes, 0);
  memcpy(c->blob.data(), &h, sizeof h);
  memcpy(c->blob.data() + h.off_bucket, bucket.data(), 257 * sizeof(uint16_t));
  if (!keys.empty()) memcpy(c->blob.data() + h.off_keys, keys.data(), keys.size() * sizeof(A5xKey));
  if (!ch.empty()) memcpy(c->blob.data() + h.off_choices, ch.data(), ch.size() * sizeof(A5xChoice));
  if (!blob.empty()) memcpy(c->blob.data() + h.off_blob, blob.data(), blob.size());
  // the walk's compact views (k_keyspace_thread psk_walk): one read per byte, one per key
  for (size_t k = 0; k < keys.size(); k++) {
    const uint64_t km = (uint64_t)ch[keys[k].choice_base].first4 | ((uint64_t)keys[k].klen << 32);
    memcpy(c->blob.data() + h.off_kmatch + 8 * k, &km, 8);
  }
  for (int b = 0; b < 256; b++) {
    const uint32_t v = (uint32_t)bucket[b] | ((uint32_t)bucket[b + 1] << 16);
    memcpy(c->blob.data() + h.off_bucket2 + 4 * b, &v, 4);
  }
  for (size_t i = 0; i < ch.size(); i++) {  // the planner's choice bytes, one read each
    uint64_t v = 0;
    for (uint32_t k = 0; k < ch[i].len && k < 7; k++) v |= (uint64_t)blob[ch[i].blob_off + k] << (8 * k);
    v |= (uint64_t)std::min<uint32_t>(ch[i].len, 255) << 56;
    memcpy(c->blob.data() + h.off_cval + 8 * i, &v, 8);
  }
  c->table_bytes = h.total_bytes;
  return A5X_OK;
}

// the compiled table's keys all start on UTF-8 lead (or ASCII) bytes (A5xTableHdr::lead_only)
bool table_lead_only(const a5x_ctx* c) {
  return c->blob.size() >= sizeof(A5xTableHdr) && ((const A5xTableHdr*)c->blob.data())->lead_only != 0 &&
         !getenv("A5X_NO_UTF_WALK");
}

int upload_table(a5x_ctx* c) {
  if (c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (c->table.keys.empty()) return fail(c, A5X_E_NOTABLE, "no substitution table loaded");
  if (!c->table_dirty) return A5X_OK;
  int rc = compile_table(c);
  if (rc) return rc;
  if (c->d_table_cap < c->blob.size()) {
    if (c->d_table) (void)hipFree(c->d_table);
    c->d_table = nullptr;
    HIPCHK(c, hipMalloc((void**)&c->d_table, c->blob.size()));
    c->d_table_cap = c->blob.size();
  }
  HIPCHK(c, hipMemcpyAsync(c->d_table, c->blob.data(), c->blob.size(), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->table_dirty = false;
  return A5X_OK;
}

int check_mode(a5x_ctx* c, int mode) {
  if (mode < 0 || mode > 3) return fail(c, A5X_E_ARG, "bad mode %d", mode);
  return A5X_OK;
}

int decode_dev_err(a5x_ctx* c, uint32_t e) {
  if (!e) return A5X_OK;
  if (e & 32u) {
    uint64_t d[8] = {0};
    (void)hipMemcpy(d, c->d_scalars + 16, sizeof d, hipMemcpyDeviceToHost);
    return fail(c, A5X_E_HIP,
                "device bounds guard tripped: code %llu ctx {%llu, %llu, %llu, %llu} block %llu thread %llu",
                (unsigned long long)d[0], (unsigned long long)d[1], (unsigned long long)d[2],
                (unsigned long long)d[3], (unsigned long long)d[4], (unsigned long long)d[5],
                (unsigned long long)d[6]);
  }
  if (e & 128u)
    return fail(c, A5X_E_BOUNDS,
                "panic: runtime error: slice bounds out of range (processWordReverse, main.go:255: a negative "
                "actualStart from the running offset)");
  if (e & 64u)
    return fail(c, A5X_E_UNSUPPORTED,
                "a word exceeds the -r/-s engine limits (length <= %d B, <= %d patterns/positions, DP <= %d "
                "entries, <= %d keys)", A5X_M_LMAX, A5X_M_NMAX, A5X_M_DPMAX, A5X_MTAB_KEYS_MAX);
  if (e & 256u)
    return fail(c, A5X_E_UNSUPPORTED, "a -r/-s candidate is longer than %d bytes (device limit)", A5X_M_CBUF - 1);
  if (e & 2u) return fail(c, A5X_E_OVERFLOW, "a word's keyspace overflows 64 bits");
  if (e & 16u) return fail(c, A5X_E_OVERFLOW, "batch keyspace overflows 64 bits");
  if (e & 4u)
    return fail(c, A5X_E_UNSUPPORTED,
                "a word with candidates exceeds the device limits (length %d B, %d matches, min(max,matches) "
                "<= 63 substitutions unless the window is free, DP (events+1) x (min(max,matches)+1) <= %u, "
                "candidates <= %u B)", A5X_LMAX_G, A5X_MLMAX_G, (unsigned)A5X_DPENT_G, (unsigned)A5X_RING_G - 16u);
  return fail(c, A5X_E_HIP, "device consistency error 0x%x", e);
}

// words with overlapping keys (or other irregular shapes) whose FAST records go to
// fixed slots after the tile regions: this many slots at first (a batch with more complex
// words grows them and runs its keyspace again, run_keyspace)
uint32_t ks_cplx_cap(uint64_t nw) { return (uint32_t)std::min<uint64_t>(nw / 16 + 1024, 1u << 22); }

struct Batch {  // device-side per-batch state after keyspace
  uint64_t total_cands = 0, total_bytes = 0;
  uint32_t nbig = 0, nslow = 0;
  uint32_t nglob = 0;  // pass G words (on the BIG list, expanded by k_expand_g)
  bool rfast = false;  // -r / -s / -s -r: FAST words probed by k_keyspace_thread (k_expand_fast)
  uint64_t nmode = 0;  // -r / -s / -s -r: words left to the mode engine (0: no mode-item launch)
  bool virt = false;   // -s / -s -r: virtual words present; k_expand_fast runs on the virtual list
  uint64_t nv = 0;     // its entries
  const uint64_t* cand_off = nullptr;
  const uint64_t* byte_off = nullptr;
};

// keyspace -> flags, per-word counts/bytes, exclusive scans (synchronises once)
int run_keyspace(a5x_ctx* c, const uint8_t* d_words, const uint64_t* d_woff, uint64_t nw, int mn, int mx,
                 uint64_t* d_cand_off, uint64_t* d_byte_off, hipStream_t st, Batch* B, bool timed) {
  int rc;
  if ((rc = upload_table(c))) return rc;
  if (nw > 0xffffffffull) return fail(c, A5X_E_ARG, "batch of %llu words (max 2^32-1)", (unsigned long long)nw);
  // FAST record slots of the complex words (k_keyspace_cplx): enough for every one of them,
  // so whether a word is FAST (and how its candidates are numbered) never depends on how
  // many complex words share its batch; u32 record offsets bound the whole record area
  const uint64_t ccap = std::min<uint64_t>(nw + 1, std::max<uint64_t>(ks_cplx_cap(nw), c->cplx_need));
  if (((nw + FW_TILE - 1) / FW_TILE) * (uint64_t)FW_TILE_REC + ccap * FW_RMAX > 0xffffffffull)
    return fail(c, A5X_E_ARG, "batch of %llu words is too large for one call (FAST record index; split it)",
                (unsigned long long)nw);
  if ((rc = grow(c, c->count, nw + 1)) || (rc = grow(c, c->bytes, nw + 1)) || (rc = grow(c, c->flags, nw + 1)) ||
      (rc = grow(c, c->defer, nw + 1)) || (rc = grow(c, c->scan_tmp, a5x_scan_tmp_elems(nw + 1) + 16)) ||
      (rc = grow(c, c->roff, nw + 1)) || (rc = grow(c, c->cplx, nw + 1)) ||
      (rc = grow(c, c->slow_list, nw + 1)) || (rc = grow(c, c->big_list, nw + 1)) || (rc = grow(c, c->glob, nw + 1)) ||
      (rc = grow(c, c->rec, ((nw + FW_TILE - 1) / FW_TILE) * (uint64_t)FW_TILE_REC + ccap * FW_RMAX + 2)))
    return rc;
  if (!d_cand_off) {
    if ((rc = grow(c, c->cand_off, nw + 1))) return rc;
    d_cand_off = c->cand_off.p;
  }
  if (!d_byte_off) {
    if ((rc = grow(c, c->byte_off, nw + 1))) return rc;
    d_byte_off = c->byte_off.p;
  }
  if (timed) HIPCHK(c, hipEventRecord(c->ev[0], st));
  HIPCHK(c, hipMemsetAsync(c->d_scalars, 0, 128, st));  // scalars + guard debug record
  A5xKsLaunch K;
  memset(&K, 0, sizeof K);
  if (nw > 0) {
    K.table = c->d_table; K.table_bytes = c->table_bytes; K.words = d_words; K.woff = d_woff; K.nw = nw;
    K.mn = mn; K.mx = mx; K.count = c->count.p; K.bytes = c->bytes.p; K.flags = c->flags.p;
    K.defer_list = c->defer.p; K.defer_n = c->d_scalars; K.nbig = c->d_scalars + 1; K.err = c->d_scalars + 2;
    K.hiflag = table_lead_only(c) ? c->d_scalars + 8 : nullptr;
    K.nslow = c->d_scalars + 3;
    K.slow_list = c->slow_list.p; K.big_list = c->big_list.p;
    K.rec = c->rec.p; K.roff = c->roff.p;
    K.cplx_list = c->cplx.p; K.cplx_n = c->d_scalars + 4; K.cplx_cap = (uint32_t)ccap;
    K.cplx_base = ((nw + FW_TILE - 1) / FW_TILE) * (uint64_t)FW_TILE_REC;
    K.defer_blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(nw, (uint64_t)c->cus * 4));
    K.glob_list = c->glob.p; K.glob_n = c->d_scalars + 7;
    HIPCHK(c, a5x_launch_keyspace(K, st));
    HIPCHK(c, a5x_launch_scan(c->count.p, c->bytes.p, nw, d_cand_off, d_byte_off, c->scan_tmp.p,
                              c->d_scalars + 2, st));
    HIPCHK(c, hipMemcpyAsync(c->h_totals, d_cand_off + nw, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(c->h_totals + 1, d_byte_off + nw, 8, hipMemcpyDeviceToHost, st));
  } else {
    HIPCHK(c, hipMemsetAsync(d_cand_off, 0, 8, st));
    HIPCHK(c, hipMemsetAsync(d_byte_off, 0, 8, st));
    c->h_totals[0] = c->h_totals[1] = 0;
  }
  HIPCHK(c, hipMemcpyAsync(c->h_scalars, c->d_scalars, 32, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  if (nw > 0 && c->h_scalars[4] > ccap) {
    // more complex words than record slots: room for all of them, and the keyspace again
    c->cplx_need = c->h_scalars[4];
    return run_keyspace(c, d_words, d_woff, nw, mn, mx, d_cand_off, d_byte_off, st, B, timed);
  }
  if (nw > 0 && c->h_scalars[2] == 0 && c->h_scalars[7] > 0) {
    // pass G: words beyond the pass-B LDS budget are sized in HBM scratch slots (their
    // counts were 0 in the first scan), then the scan runs again
    if (!c->gscr) {
      const size_t gb = (size_t)A5X_G_SLOTS * a5x_gslot_bytes();
      HIPCHK(c, hipMalloc((void**)&c->gscr, gb));
      HIPCHK(c, hipMemsetAsync(c->gscr, 0, gb, st));  // the rings start (and stay) zero
    }
    K.gscr = c->gscr; K.gslots = A5X_G_SLOTS;
    HIPCHK(c, a5x_launch_keyspace_g(K, st));
    HIPCHK(c, a5x_launch_scan(c->count.p, c->bytes.p, nw, d_cand_off, d_byte_off, c->scan_tmp.p,
                              c->d_scalars + 2, st));
    HIPCHK(c, hipMemcpyAsync(c->h_totals, d_cand_off + nw, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(c->h_totals + 1, d_byte_off + nw, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(c->h_scalars, c->d_scalars, 32, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
  }
  if ((rc = decode_dev_err(c, c->h_scalars[2]))) {
    // name the first offending word (diagnostics)
    std::vector<uint32_t> fl(nw);
    std::vector<uint64_t> wo(nw + 1);
    if (nw && hipMemcpy(fl.data(), c->flags.p, nw * 4, hipMemcpyDeviceToHost) == hipSuccess &&
        hipMemcpy(wo.data(), d_woff, (nw + 1) * 8, hipMemcpyDeviceToHost) == hipSuccess) {
      for (uint64_t i = 0; i < nw; i++)
        if (fl[i] & (A5X_WF_ERR_BIG | A5X_WF_ERR_OVF)) {
          std::string w((size_t)(wo[i + 1] - wo[i]), '\0');
          (void)hipMemcpy(&w[0], d_words + wo[i], w.size(), hipMemcpyDeviceToHost);
          char tail[160];
          snprintf(tail, sizeof tail, " [word %llu len %zu flags 0x%08x: %.40s]", (unsigned long long)i, w.size(),
                   fl[i], w.c_str());
          c->err += tail;
          break;
        }
    }
    return rc;
  }
  B->total_cands = nw ? c->h_totals[0] : 0;
  B->total_bytes = nw ? c->h_totals[1] : 0;
  B->nbig = c->h_scalars[1];
  B->nslow = c->h_scalars[3];
  B->nglob = nw ? c->h_scalars[7] : 0;
  B->cand_off = d_cand_off;
  B->byte_off = d_byte_off;
  return A5X_OK;
}

A5xExpLaunch exp_launch(a5x_ctx* c, const uint8_t* d_words, const uint64_t* d_woff, uint64_t nw, int mn, int mx,
                        const Batch& B) {
  A5xExpLaunch E;
  memset(&E, 0, sizeof E);
  E.table = c->d_table; E.table_bytes = c->table_bytes; E.words = d_words; E.woff = d_woff; E.nw = nw;
  E.cand_off = B.cand_off; E.byte_off = B.byte_off; E.flags = c->flags.p; E.chunk_w0 = c->chunk_w0.p;
  E.CH = c->chunk; E.SEG = c->seg; E.mn = mn; E.mx = mx; E.err = c->d_scalars + 2;
  E.dbg = (uint64_t*)(c->d_scalars + 16);
  E.waves_per_block = c->waves_per_block;
  E.waves_per_block_fast = c->waves_per_block_fast;
  E.rec = c->rec.p; E.roff = c->roff.p; E.rec_n = c->rec.cap;
  if (B.nglob) { E.gscr = c->gscr; E.gslots = A5X_G_SLOTS; }
  return E;
}


// ---------------------------------------------------------------------------
// -r / -s / -s -r engines (a5x_modes.hip)
// ---------------------------------------------------------------------------

// The sorted mode table of a5x_format.h (keys in Go sort.Strings order, main.go:327).
int compile_mtable(a5x_ctx* c) {
  const Table& t = c->table;
  std::vector<uint32_t> order(t.keys.size());
  for (uint32_t i = 0; i < order.size(); i++) order[i] = i;
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return t.keys[a] < t.keys[b]; });
  if (order.size() > A5X_MTAB_KEYS_MAX)
    return fail(c, A5X_E_UNSUPPORTED, "table has %zu keys (-r/-s device engines: max %d)", order.size(),
                A5X_MTAB_KEYS_MAX);
  std::vector<A5xMKey> keys;
  std::vector<A5xMVal> vals;
  std::vector<uint8_t> blob;
  std::vector<uint16_t> bucket(257, 0);
  uint32_t has_empty = 0;
  for (uint32_t i : order) {
    const std::string& k = t.keys[i];
    if (k.empty()) has_empty = 1;  // sorts first: key 0
    else bucket[(uint8_t)k[0] + 1]++;
    A5xMKey K;
    memset(&K, 0, sizeof K);
    if (k.size() > 65535 || t.vals[i].size() > 65535) return fail(c, A5X_E_UNSUPPORTED, "table key too large");
    K.key_off = (uint32_t)blob.size();
    K.klen = (uint16_t)k.size();
    K.nvals = (uint16_t)t.vals[i].size();
    K.val_base = (uint32_t)vals.size();
    blob.insert(blob.end(), k.begin(), k.end());
    for (auto& v : t.vals[i]) {
      A5xMVal V;
      V.off = (uint32_t)blob.size();
      V.len = (uint32_t)v.size();
      blob.insert(blob.end(), v.begin(), v.end());
      vals.push_back(V);
    }
    keys.push_back(K);
  }
  // static per-key facts (key_pos_facts) for the lane-per-word -s / -s -r keyspace
  for (size_t i = 0; i < order.size(); i++)
    keys[i].pad = key_pos_facts(t, t.keys[order[i]], t.vals[order[i]]);
  bucket[0] = (uint16_t)has_empty;
  for (int b = 0; b < 256; b++) bucket[b + 1] += bucket[b];
  auto al16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  A5xMHdr h;
  memset(&h, 0, sizeof h);
  h.magic = A5X_MTAB_MAGIC;
  h.nkeys = (uint32_t)keys.size();
  h.nvals = (uint32_t)vals.size();
  h.has_empty = has_empty;
  h.off_bucket = sizeof(A5xMHdr);
  h.off_keys = (uint32_t)al16(h.off_bucket + 257 * sizeof(uint16_t));
  h.off_vals = (uint32_t)al16(h.off_keys + keys.size() * sizeof(A5xMKey));
  h.off_blob = (uint32_t)al16(h.off_vals + vals.size() * sizeof(A5xMVal));
  const size_t total = al16(h.off_blob + blob.size() + 8);
  if (total > A5X_MTAB_LDS_MAX)
    return fail(c, A5X_E_UNSUPPORTED, "mode table is %zu bytes (-r/-s LDS staging max %d)", total,
                A5X_MTAB_LDS_MAX);
  h.total_bytes = (uint32_t)total;
  c->mblob.assign(total, 0);
  memcpy(c->mblob.data(), &h, sizeof h);
  memcpy(c->mblob.data() + h.off_bucket, bucket.data(), 257 * sizeof(uint16_t));
  if (!keys.empty()) memcpy(c->mblob.data() + h.off_keys, keys.data(), keys.size() * sizeof(A5xMKey));
  if (!vals.empty()) memcpy(c->mblob.data() + h.off_vals, vals.data(), vals.size() * sizeof(A5xMVal));
  if (!blob.empty()) memcpy(c->mblob.data() + h.off_blob, blob.data(), blob.size());
  c->mtab_bytes = (uint32_t)total;
  return A5X_OK;
}

int upload_mtable(a5x_ctx* c) {
  if (c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (c->table.keys.empty()) return fail(c, A5X_E_NOTABLE, "no substitution table loaded");
  if (!c->mtable_dirty) return A5X_OK;
  int rc = compile_mtable(c);
  if (rc) return rc;
  if (c->d_mtab_cap < c->mblob.size()) {
    if (c->d_mtab) (void)hipFree(c->d_mtab);
    c->d_mtab = nullptr;
    HIPCHK(c, hipMalloc((void**)&c->d_mtab, c->mblob.size()));
    c->d_mtab_cap = c->mblob.size();
  }
  HIPCHK(c, hipMemcpyAsync(c->d_mtab, c->mblob.data(), c->mblob.size(), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->mtable_dirty = false;
  return A5X_OK;
}

A5xModeLaunch mode_launch(a5x_ctx* c, const uint8_t* d_words, const uint64_t* d_woff, uint64_t nw, int mode,
                          int mn, int mx, bool rfast = false, bool virt = false) {
  A5xModeLaunch M;
  memset(&M, 0, sizeof M);
  M.rfast = rfast ? 1 : 0;
  if (rfast) { M.rec = c->rec.p; M.roff = c->roff.p; }
  if (virt) {
    M.vpre = c->vpre.p; M.vcand_off = c->vcand_off.p; M.vbyte_off = c->vbyte_off.p;
    M.vroff = c->vroff.p; M.vrec = c->vrec2.p;
  }
  M.mtab = c->d_mtab; M.mtab_bytes = c->mtab_bytes; M.words = d_words; M.woff = d_woff; M.nw = nw;
  M.mode = mode; M.mn = mn; M.mx = mx; M.SEG = c->mseg;
  M.count = c->count.p; M.nseg = c->m_nseg.p; M.flags = c->flags.p;
  M.wbytes = c->bytes.p;  // (scratch until k_mode_wordbytes writes the per-word bytes)
  M.seg_off = c->m_seg_off.p; M.item_w = c->m_item_w.p; M.nitems = c->m_items;
  M.seg_bytes = c->m_seg_bytes.p; M.seg_boff = c->m_seg_boff.p; M.item_fl = c->m_item_fl.p;
  M.cand_begin = 0; M.cand_end = ~0ull;
  M.err = c->d_scalars + 2;
  M.glob_list = c->glob.p; M.glob_n = c->d_scalars + 7;
  if (c->m_nglob) { M.gscr = c->mgscr; M.gslots = A5X_G_SLOTS; }
  return M;
}

// The virtual word list of a -s / -s -r batch with virtual words (k_keyspace_vsub): every
// word one entry, a virtual word one per sub-word, records in list order (copied, or written
// from a fixed-width word's descriptor); the chunk -> first entry map of k_expand_fast over it.
// byte_off null: no output layout (fused digest).  Synchronises once.
int build_virtual(a5x_ctx* c, uint64_t nw, const uint8_t* d_words, const uint64_t* d_woff, int mode, int mn,
                  const uint64_t* d_cand_off, const uint64_t* d_byte_off, hipStream_t st, Batch* B) {
  int rc;
  if ((rc = grow(c, c->vpre, nw + 1)) || (rc = grow(c, c->vrpre, nw + 1))) return rc;
  HIPCHK(c, a5x_launch_vwords_sizes(c->flags.p, d_cand_off, nw, c->vn.p, c->vrsz.p, st));
  HIPCHK(c, a5x_launch_scan(c->vn.p, c->vrsz.p, nw, c->vpre.p, c->vrpre.p, c->scan_tmp.p, c->d_scalars + 2, st));
  HIPCHK(c, hipMemcpyAsync(c->h_totals + 4, c->vpre.p + nw, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipMemcpyAsync(c->h_totals + 5, c->vrpre.p + nw, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  const uint64_t nv = nw + c->h_totals[4], nrec = c->h_totals[5];
  if (nv > 0xffffffffull || nrec + 4 > 0xffffffffull)
    return fail(c, A5X_E_ARG, "batch of %llu words is too large for one -s call (virtual word list)",
                (unsigned long long)nw);
  if ((rc = grow(c, c->vcand_off, nv + 1)) || (rc = grow(c, c->vbyte_off, nv + 1)) ||
      (rc = grow(c, c->vflags, nv + 1)) || (rc = grow(c, c->vroff, nv + 1)) || (rc = grow(c, c->vmap, nv + 1)) ||
      (rc = grow(c, c->vobase, nv + 1)) || (rc = grow(c, c->vrec2, nrec + 4)))
    return rc;
  A5xVwLaunch V;
  V.flags = c->flags.p; V.cand_off = d_cand_off; V.byte_off = d_byte_off; V.roff = c->roff.p; V.rec = c->rec.p;
  V.vrec = c->vrec.p; V.vpre = c->vpre.p; V.vrpre = c->vrpre.p; V.nw = nw;
  V.vcand_off = c->vcand_off.p; V.vbyte_off = c->vbyte_off.p; V.vflags = c->vflags.p; V.vroff = c->vroff.p;
  V.vmap = c->vmap.p; V.vobase = c->vobase.p; V.vrec2 = c->vrec2.p;
  V.table = c->d_table; V.table_bytes = c->table_bytes; V.rmode = mode; V.rcmin = mn > 0 ? 1u : 0u;
  V.words = d_words; V.woff = d_woff;
  HIPCHK(c, a5x_launch_vwords_fill(V, st));
  if (B->total_cands) {
    const uint64_t nchunks = (B->total_cands + c->chunk - 1) / c->chunk;
    if ((rc = grow(c, c->chunk_w0, nchunks + 1))) return rc;
    HIPCHK(c, a5x_launch_plan(c->vcand_off.p, nv, c->chunk, c->chunk_w0.p, st));
  }
  B->virt = true;
  B->nv = nv;
  return A5X_OK;
}

// k_expand_fast over a -r / -s / -s -r batch's FAST words (the virtual word list when the
// batch has virtual words)
A5xExpLaunch exp_launch_mode(a5x_ctx* c, const uint8_t* d_words, const uint64_t* d_woff, uint64_t nw, int mn, int mx,
                             const Batch& B) {
  A5xExpLaunch E = exp_launch(c, d_words, d_woff, nw, mn, mx, B);
  if (B.virt) {
    E.nw = B.nv; E.cand_off = c->vcand_off.p; E.byte_off = c->vbyte_off.p; E.flags = c->vflags.p;
    E.roff = c->vroff.p; E.rec = c->vrec2.p; E.rec_n = c->vrec2.cap; E.vmap = c->vmap.p; E.vobase = c->vobase.p;
  }
  return E;
}

// Keyspace of the -r / -s / -s -r engines: per-word counts (DP), items of mseg
// candidates, a length pass over every item (output bytes are not closed-form under
// sequential strings.ReplaceAll), and the scans.  Synchronises twice.
// lengths = false (the fused digest): counts and items only -- no length pass, no
// output layout (B->total_bytes = 0).
int run_keyspace_mode(a5x_ctx* c, const uint8_t* d_words, const uint64_t* d_woff, uint64_t nw, int mode, int mn,
                      int mx, uint64_t* d_cand_off, uint64_t* d_byte_off, hipStream_t st, Batch* B, bool timed,
                      bool lengths = true) {
  int rc;
  if ((rc = upload_mtable(c))) return rc;
  if (nw > 0xffffffffull) return fail(c, A5X_E_ARG, "batch of %llu words (max 2^32-1)", (unsigned long long)nw);
  // -r with min < 0: the subCount loop (main.go:238) reaches k = min < 0 whenever it runs
  // at all (min(max, n) >= min, i.e. max >= min), and generateCombinations(n, k < 0)
  // recurses until the goroutine stack overflows (main.go:263-281), which kills the
  // reference process on the first word.
  if (mode == A5X_MODE_REVERSE && mn < 0 && mx >= mn && nw > 0)
    return fail(c, A5X_E_BOUNDS,
                "fatal error: stack overflow (generateCombinations with k < 0, main.go:273; --table-min %d)", mn);
  if ((rc = grow(c, c->count, nw + 1)) || (rc = grow(c, c->bytes, nw + 1)) || (rc = grow(c, c->flags, nw + 1)) ||
      (rc = grow(c, c->m_nseg, nw + 1)) || (rc = grow(c, c->m_seg_off, nw + 1)) ||
      (rc = grow(c, c->glob, nw + 1)) || (rc = grow(c, c->scan_tmp, a5x_scan_tmp_elems(nw + 1) + 16)))
    return rc;
  c->m_nglob = 0;
  if (!d_cand_off) {
    if ((rc = grow(c, c->cand_off, nw + 1))) return rc;
    d_cand_off = c->cand_off.p;
  }
  if (!d_byte_off) {
    if ((rc = grow(c, c->byte_off, nw + 1))) return rc;
    d_byte_off = c->byte_off.p;
  }
  if (timed) HIPCHK(c, hipEventRecord(c->ev[0], st));
  HIPCHK(c, hipMemsetAsync(c->d_scalars, 0, 128, st));
  B->cand_off = d_cand_off;
  B->byte_off = d_byte_off;
  B->nbig = B->nslow = 0;
  B->rfast = false;
  B->virt = false;
  B->nv = 0;
  if (nw == 0) {
    HIPCHK(c, hipMemsetAsync(d_cand_off, 0, 8, st));
    HIPCHK(c, hipMemsetAsync(d_byte_off, 0, 8, st));
    HIPCHK(c, hipStreamSynchronize(st));
    B->total_cands = B->total_bytes = 0;
    c->m_items = 0;
    return A5X_OK;
  }
  // FAST probe (a5x_kernels.hip mode_unit): -r words with pairwise disjoint positions whose
  // subs[0] keep the key lengths, -s / -s -r words whose every pattern occurs once and is
  // statically positional, go to the FAST path: the default keyspace kernel plans them
  // (count, bytes, record; flags & A5X_WF_FAST), the mode-engine kernels skip them, and
  // k_expand_fast (k_expand_fast_md5 / _ntlm in the fused digest) writes them beside the
  // mode engine's items -- every path numbers a word's candidates the same way.  The other
  // words are listed for the mode engine.  (An empty key makes "" a pattern of every -s word.)
  const bool has_empty = ((const A5xMHdr*)c->mblob.data())->has_empty != 0;
  bool rfast = mx >= 1 && mn <= 1 && !getenv("A5X_NO_RFAST") &&
               (mode == A5X_MODE_REVERSE || ((mode == A5X_MODE_SUBALL || mode == A5X_MODE_SUBALL_REVERSE) && !has_empty));
  if (rfast && upload_table(c) != A5X_OK) {  // (a table the default engine refuses: mode engine only)
    rfast = false;
    c->err.clear();
  }
  B->rfast = rfast;
  // -s / -s -r: radix positional words counted lane per word (k_mode_count_thread) over the
  // words the probe left; the wave kernel k_mode_count only for the words it lists
  const bool mct = (mode == A5X_MODE_SUBALL || mode == A5X_MODE_SUBALL_REVERSE) && mx >= 0 && !has_empty &&
                   !getenv("A5X_NO_MCT");
  if ((rfast || mct) && ((rc = grow(c, c->m_cl, nw + 1)) || (rc = grow(c, c->m_cl2, nw + 1)))) return rc;
  // -s / -s -r words the probe refused for repeated patterns: split into FAST sub-words
  // (k_keyspace_vsub) before the mode engine counts the rest
  const bool vsub = rfast && mct && mode != A5X_MODE_REVERSE && !getenv("A5X_NO_VSUB");
  const uint64_t vcap = std::min<uint64_t>(0xfffffff0ull, std::max<uint64_t>(nw * 64 + 4096, c->vrec_need));
  if (vsub && ((rc = grow(c, c->m_vl, nw + 1)) || (rc = grow(c, c->vn, nw + 1)) || (rc = grow(c, c->vrsz, nw + 1)) ||
               (rc = grow(c, c->vrec, vcap + 2)) || (rc = grow(c, c->vocc, 16 * (nw + 1)))))
    return rc;
  // (the probe's overflow slots: words a keyspace tile could not decide, k_keyspace_rprobe)
  const uint64_t rtiles = ((nw + FW_TILE - 1) / FW_TILE) * (uint64_t)FW_TILE_REC;
  const uint64_t rcap = std::min<uint64_t>(nw, std::max<uint64_t>(ks_cplx_cap(nw), c->rov_need));
  if (rfast) {
    if (rtiles + rcap * FW_RMAX > 0xffffffffull)  // (u32 record offsets)
      return fail(c, A5X_E_ARG, "batch of %llu words is too large for one -r/-s call (FAST record index)",
                  (unsigned long long)nw);
    if ((rc = grow(c, c->roff, nw + 1)) || (rc = grow(c, c->cplx, nw + 1)) ||
        (rc = grow(c, c->rec, rtiles + rcap * FW_RMAX + 2)))
      return rc;
    A5xKsLaunch K;
    memset(&K, 0, sizeof K);
    K.table = c->d_table; K.table_bytes = c->table_bytes; K.words = d_words; K.woff = d_woff; K.nw = nw;
    K.mn = mn; K.mx = mx; K.count = c->count.p; K.bytes = c->bytes.p; K.flags = c->flags.p;
    K.err = c->d_scalars + 2; K.rec = c->rec.p; K.roff = c->roff.p;
    K.rmode = mode; K.rcmin = mn > 0 ? 1u : 0u; K.rnseg = c->m_nseg.p; K.rseg = c->mseg;
    K.defer_list = c->m_cl.p; K.defer_n = c->d_scalars + 12;
    K.cplx_list = c->cplx.p; K.cplx_n = c->d_scalars + 14; K.cplx_cap = (uint32_t)rcap; K.cplx_base = rtiles;
    K.defer_blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((nw + 255) / 256, (uint64_t)c->cus * 2));
    K.vocc = vsub ? c->vocc.p : nullptr;
    K.hiflag = table_lead_only(c) ? c->d_scalars + 8 : nullptr;
    HIPCHK(c, a5x_launch_keyspace(K, st));
    if (vsub) {
      K.vout_list = c->m_vl.p; K.vout_n = c->d_scalars + 15;
      K.vn = c->vn.p; K.vrsz = c->vrsz.p; K.vrec = c->vrec.p;
      K.vrec_n = (uint64_t*)(c->d_scalars + 10); K.vrec_cap = vcap;
      if (!getenv("A5X_VSUB_LARGE_ONLY")) {  // (m_cl2 is free until k_mode_count_thread below)
        K.vlong_list = c->m_cl2.p; K.vlong_n = c->d_scalars + 9;
      }
      HIPCHK(c, a5x_launch_vsub(K, st));
    }
  }
  A5xModeLaunch M = mode_launch(c, d_words, d_woff, nw, mode, mn, mx, rfast);
  if (mct) {
    M.in_list = vsub ? c->m_vl.p : rfast ? c->m_cl.p : nullptr;
    M.in_n = vsub ? c->d_scalars + 15 : rfast ? c->d_scalars + 12 : nullptr;
    M.cl_list = rfast ? c->m_cl2.p : c->m_cl.p;
    M.cl_n = c->d_scalars + (rfast ? 13 : 12);
    HIPCHK(c, a5x_launch_mode_count_thread(M, st));
  } else if (rfast) {  // k_mode_count only over the words the probe left to the mode engine
    M.cl_list = c->m_cl.p;
    M.cl_n = c->d_scalars + 12;
  }
  HIPCHK(c, a5x_launch_mode_count(M, st));
  HIPCHK(c, a5x_launch_scan(c->count.p, c->m_nseg.p, nw, d_cand_off, c->m_seg_off.p, c->scan_tmp.p,
                            c->d_scalars + 2, st));
  HIPCHK(c, hipMemcpyAsync(c->h_totals, d_cand_off + nw, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipMemcpyAsync(c->h_totals + 1, c->m_seg_off.p + nw, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipMemcpyAsync(c->h_scalars, c->d_scalars, 64, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  if (rfast && c->h_scalars[14] > rcap) {
    // more undecided words than overflow slots: grow to fit them all and run again (the
    // undecided tail was left uncounted, so nothing of this pass is used)
    c->rov_need = c->h_scalars[14];
    return run_keyspace_mode(c, d_words, d_woff, nw, mode, mn, mx, d_cand_off, d_byte_off, st, B, timed, lengths);
  }
  uint64_t vused = 0;
  if (vsub) memcpy(&vused, c->h_scalars + 10, 8);
  if (vsub && vused > vcap) {
    // more sub-word records than room: grow to fit them all and run again (words past
    // the room were left undecided)
    if (vused > 0xfffffff0ull)
      return fail(c, A5X_E_ARG, "batch of %llu words is too large for one -s call (sub-word records)",
                  (unsigned long long)nw);
    c->vrec_need = vused;
    return run_keyspace_mode(c, d_words, d_woff, nw, mode, mn, mx, d_cand_off, d_byte_off, st, B, timed, lengths);
  }
  B->nmode = vsub ? c->h_scalars[15] : rfast ? c->h_scalars[12] : nw;
  if (vsub && getenv("A5X_VSUB_DEBUG")) {  // (diagnostics: what the split leaves to the mode engine)
    fprintf(stderr, "[vsub] words %llu probe-left %u split-left %u vrec %llu\n", (unsigned long long)nw,
            c->h_scalars[12], c->h_scalars[15], (unsigned long long)vused);
    const uint32_t k = std::min<uint32_t>(c->h_scalars[15], 24);
    std::vector<uint32_t> li(k);
    std::vector<uint64_t> wo(nw + 1);
    if (k && hipMemcpy(li.data(), c->m_vl.p, 4 * k, hipMemcpyDeviceToHost) == hipSuccess &&
        hipMemcpy(wo.data(), d_woff, 8 * (nw + 1), hipMemcpyDeviceToHost) == hipSuccess)
      for (uint32_t x : li) {
        std::string s((size_t)(wo[x + 1] - wo[x]), '\0');
        (void)hipMemcpy(&s[0], d_words + wo[x], s.size(), hipMemcpyDeviceToHost);
        fprintf(stderr, "[vsub]   left: %s\n", s.c_str());
      }
  }
  if (c->h_scalars[2] == 0 && c->h_scalars[7] > 0) {
    // mode pass G: words longer than the LDS engines take are counted in HBM scratch
    // slots (their counts were 0 in the first scan), then the scan runs again
    if (!c->mgscr) {
      HIPCHK(c, hipMalloc((void**)&c->mgscr, (size_t)A5X_G_SLOTS * a5x_mode_gslot_bytes()));
    }
    c->m_nglob = c->h_scalars[7];
    M = mode_launch(c, d_words, d_woff, nw, mode, mn, mx, rfast);
    HIPCHK(c, a5x_launch_mode_count_g(M, st));
    HIPCHK(c, a5x_launch_scan(c->count.p, c->m_nseg.p, nw, d_cand_off, c->m_seg_off.p, c->scan_tmp.p,
                              c->d_scalars + 2, st));
    HIPCHK(c, hipMemcpyAsync(c->h_totals, d_cand_off + nw, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(c->h_totals + 1, c->m_seg_off.p + nw, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(c->h_scalars, c->d_scalars, 32, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
  }
  auto name_word = [&]() {
    std::vector<uint32_t> fl(nw);
    std::vector<uint64_t> wo(nw + 1);
    if (hipMemcpy(fl.data(), c->flags.p, nw * 4, hipMemcpyDeviceToHost) == hipSuccess &&
        hipMemcpy(wo.data(), d_woff, (nw + 1) * 8, hipMemcpyDeviceToHost) == hipSuccess) {
      for (uint64_t i = 0; i < nw; i++)
        if (fl[i] & (A5X_WF_ERR_BIG | A5X_WF_ERR_OVF)) {
          std::string w((size_t)(wo[i + 1] - wo[i]), '\0');
          (void)hipMemcpy(&w[0], d_words + wo[i], w.size(), hipMemcpyDeviceToHost);
          char tail[160];
          snprintf(tail, sizeof tail, " [word %llu len %zu: %.40s]", (unsigned long long)i, w.size(), w.c_str());
          c->err += tail;
          break;
        }
    }
  };
  if ((rc = decode_dev_err(c, c->h_scalars[2]))) {
    name_word();
    return rc;
  }
  B->total_cands = c->h_totals[0];
  const uint64_t items = c->h_totals[1];
  c->m_items = items;
  if ((rc = grow(c, c->m_item_w, items + 1)) || (rc = grow(c, c->m_seg_bytes, items + 1)) ||
      (rc = grow(c, c->m_item_fl, items + 1)) ||
      (rc = grow(c, c->m_seg_boff, items + 1)) || (rc = grow(c, c->m_tmp, items + 1)) ||
      (rc = grow(c, c->scan_tmp, a5x_scan_tmp_elems(items + 1) + 16)))
    return rc;
  M = mode_launch(c, d_words, d_woff, nw, mode, mn, mx, rfast);
  M.cand_off = d_cand_off;
  M.item_begin = 0;
  M.item_end = items;
  if (rfast && B->total_cands) {  // chunk -> first word map for k_expand_fast
    const uint64_t nchunks = (B->total_cands + c->chunk - 1) / c->chunk;
    if ((rc = grow(c, c->chunk_w0, nchunks + 1))) return rc;
    HIPCHK(c, a5x_launch_plan(d_cand_off, nw, c->chunk, c->chunk_w0.p, st));
  }
  if (items) HIPCHK(c, a5x_launch_plan(c->m_seg_off.p, nw, 1, c->m_item_w.p, st));
  if (!lengths) {
    HIPCHK(c, hipMemcpyAsync(c->h_scalars, c->d_scalars, 16, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if ((rc = decode_dev_err(c, c->h_scalars[2]))) return rc;
    B->total_bytes = 0;
    return vused ? build_virtual(c, nw, d_words, d_woff, mode, mn, d_cand_off, nullptr, st, B) : A5X_OK;
  }
  if (items) HIPCHK(c, a5x_launch_mode_items(M, 0, st));
  if (items)
    HIPCHK(c, a5x_launch_scan(c->m_seg_bytes.p, c->m_seg_bytes.p, items, c->m_seg_boff.p, c->m_tmp.p,
                              c->scan_tmp.p, c->d_scalars + 2, st));
  else
    HIPCHK(c, hipMemsetAsync(c->m_seg_boff.p, 0, 8, st));
  HIPCHK(c, a5x_launch_mode_wordbytes(c->m_seg_off.p, c->m_seg_boff.p, nw, d_byte_off, c->bytes.p, st));
  HIPCHK(c, hipMemcpyAsync(c->h_totals + 1, d_byte_off + nw, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipMemcpyAsync(c->h_scalars, c->d_scalars, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  if ((rc = decode_dev_err(c, c->h_scalars[2]))) return rc;
  B->total_bytes = c->h_totals[1];
  return vused ? build_virtual(c, nw, d_words, d_woff, mode, mn, d_cand_off, d_byte_off, st, B) : A5X_OK;
}

// ---------------------------------------------------------------------------
// Batch jobs: the keyspace runs once per batch (job_prepare), then any number of
// candidate ranges are located and expanded against it (job_locate, job_launch).
// ---------------------------------------------------------------------------
struct Job {
  const uint8_t* w = nullptr;
  const uint64_t* wo = nullptr;
  uint64_t nw = 0;
  int mode = 0, mn = 0, mx = 0;
  hipStream_t st = nullptr;
  bool lengths = true;  // -r / -s engines: output layout wanted (false: the fused digest)
  Batch B;
};

// [cb, ce) global candidates <-> output bytes [b0, b1); -r/-s engines: items [i0, i1)
struct Range {
  uint64_t cb, ce, b0, b1, i0, i1;
};

int job_prepare(a5x_ctx* c, Job& J, uint64_t* d_cand_off, uint64_t* d_byte_off, bool timed) {
  int rc;
  if (J.mode != A5X_MODE_DEFAULT)
    return run_keyspace_mode(c, J.w, J.wo, J.nw, J.mode, J.mn, J.mx, d_cand_off, d_byte_off, J.st, &J.B, timed,
                             J.lengths);
  if ((rc = run_keyspace(c, J.w, J.wo, J.nw, J.mn, J.mx, d_cand_off, d_byte_off, J.st, &J.B, timed))) return rc;
  if (J.B.total_cands) {  // chunk -> first word map, consumed by every range's k_expand_fast
    const uint64_t nchunks = (J.B.total_cands + c->chunk - 1) / c->chunk;
    if ((rc = grow(c, c->chunk_w0, nchunks + 1))) return rc;
    HIPCHK(c, a5x_launch_plan(J.B.cand_off, J.nw, c->chunk, c->chunk_w0.p, J.st));
  }
  return A5X_OK;
}

int job_check(a5x_ctx* c, const Job& J) {
  HIPCHK(c, hipMemcpyAsync(c->h_scalars, c->d_scalars, 16, hipMemcpyDeviceToHost, J.st));
  HIPCHK(c, hipStreamSynchronize(J.st));
  return decode_dev_err(c, c->h_scalars[2]);
}

// Output byte (and -r/-s item) positions of global candidate indices q[0..n) (sorted or
// not); synchronises.  res[3 i] = byte offset, [3 i + 1] = item, [3 i + 2] = index in item.
int job_locate(a5x_ctx* c, const Job& J, const std::vector<uint64_t>& q, std::vector<uint64_t>& res) {
  int rc;
  const uint32_t n = (uint32_t)q.size();
  res.assign(3 * (size_t)n, 0);
  if (!n) return A5X_OK;
  if ((rc = grow(c, c->loc_q, n)) || (rc = grow(c, c->loc_r, 3 * (size_t)n))) return rc;
  HIPCHK(c, hipMemcpyAsync(c->loc_q.p, q.data(), 8 * (size_t)n, hipMemcpyHostToDevice, J.st));
  if (J.mode != A5X_MODE_DEFAULT) {
    A5xModeLaunch M = mode_launch(c, J.w, J.wo, J.nw, J.mode, J.mn, J.mx, J.B.rfast, J.B.virt);
    M.cand_off = J.B.cand_off;
    HIPCHK(c, a5x_launch_mode_locate(M, c->loc_q.p, n, c->loc_r.p, J.st));
    std::vector<uint64_t> t(3 * (size_t)n);
    HIPCHK(c, hipMemcpyAsync(t.data(), c->loc_r.p, 24 * (size_t)n, hipMemcpyDeviceToHost, J.st));
    if ((rc = job_check(c, J))) return rc;
    for (uint32_t i = 0; i < n; i++) {
      res[3 * i] = t[3 * i + 2];
      res[3 * i + 1] = t[3 * i];
      res[3 * i + 2] = t[3 * i + 1];
    }
    return A5X_OK;
  }
  A5xExpLaunch E = exp_launch(c, J.w, J.wo, J.nw, J.mn, J.mx, J.B);
  HIPCHK(c, a5x_launch_locate(E, c->loc_q.p, n, c->loc_r.p, J.st));
  std::vector<uint64_t> t(n);
  HIPCHK(c, hipMemcpyAsync(t.data(), c->loc_r.p, 8 * (size_t)n, hipMemcpyDeviceToHost, J.st));
  if ((rc = job_check(c, J))) return rc;
  for (uint32_t i = 0; i < n; i++) res[3 * i] = t[i];
  return A5X_OK;
}

Range range_of(const Job& J, uint64_t cb, uint64_t ce, const uint64_t* lb, const uint64_t* le) {
  Range R;
  R.cb = cb; R.ce = ce;
  R.b0 = lb[0]; R.b1 = le[0];
  R.i0 = lb[1];
  R.i1 = le[1] + (le[2] ? 1 : 0);
  (void)J;
  return R;
}

// Cut [0, total) into ranges of at most cap output bytes: candidate boundaries spaced for
// ~3/4 cap each, located in one call; ranges that still exceed cap are halved.
// (cb, ce: only the candidates [cb, ce) of the batch, cut into ranges the same way)
int plan_ranges(a5x_ctx* c, const Job& J, uint64_t cap, std::vector<Range>& out, uint64_t cb = 0,
                uint64_t ce = ~0ull) {
  out.clear();
  const uint64_t T = J.B.total_cands, TB = J.B.total_bytes;
  ce = std::min(ce, T);
  if (cb >= ce) return A5X_OK;
  int rc;
  uint64_t RB = TB;  // the bytes of [cb, ce)
  std::vector<uint64_t> ends;
  if (cb != 0 || ce != T) {
    if ((rc = job_locate(c, J, {cb, ce}, ends))) return rc;
    RB = ends[3] - ends[0];
  }
  if (RB <= cap) {
    if (cb == 0 && ce == T) out.push_back(Range{0, T, 0, TB, 0, J.mode != A5X_MODE_DEFAULT ? c->m_items : 0});
    else out.push_back(range_of(J, cb, ce, &ends[0], &ends[3]));
    return A5X_OK;
  }
  const uint64_t K = std::max<uint64_t>(2, (RB + cap * 3 / 4 - 1) / std::max<uint64_t>(1, cap * 3 / 4));
  std::vector<uint64_t> q(K + 1), res;
  for (uint64_t k = 0; k <= K; k++) q[k] = cb + (uint64_t)((unsigned __int128)(ce - cb) * k / K);
  if ((rc = job_locate(c, J, q, res))) return rc;
  std::vector<Range> work;
  for (uint64_t k = 0; k < K; k++)
    if (q[k + 1] > q[k]) work.push_back(range_of(J, q[k], q[k + 1], &res[3 * k], &res[3 * (k + 1)]));
  // halve oversize ranges until every range fits
  for (int pass = 0; pass < 64; pass++) {
    std::vector<uint64_t> mid;
    for (auto& R : work)
      if (R.b1 - R.b0 > cap) {
        if (R.ce - R.cb == 1)
          return fail(c, A5X_E_CAPACITY, "one candidate needs %llu bytes, the range buffer has %llu",
                      (unsigned long long)(R.b1 - R.b0), (unsigned long long)cap);
        mid.push_back(R.cb + (R.ce - R.cb) / 2);
      }
    if (mid.empty()) break;
    std::vector<uint64_t> mres;
    if ((rc = job_locate(c, J, mid, mres))) return rc;
    std::vector<Range> next;
    size_t m = 0;
    for (auto& R : work) {
      if (R.b1 - R.b0 > cap) {
        const uint64_t lb[3] = {R.b0, R.i0, 0};
        const uint64_t* lm = &mres[3 * m];
        const uint64_t le[3] = {R.b1, R.i1, 0};
        next.push_back(range_of(J, R.cb, mid[m], lb, lm));
        Range H = range_of(J, mid[m], R.ce, lm, le);
        H.i0 = lm[1];  // the half starts inside item lm[1]
        next.push_back(H);
        m++;
      } else {
        next.push_back(R);
      }
    }
    work.swap(next);
  }
  out.swap(work);
  return A5X_OK;
}

// Launch the expansion of one located range into d_out (asynchronous on J.st).
int job_launch(a5x_ctx* c, const Job& J, const Range& R, uint8_t* d_out, uint64_t out_cap) {
  int rc;
  if (R.ce <= R.cb) return A5X_OK;
  if (R.b1 - R.b0 > out_cap || (!d_out && R.b1 > R.b0))
    return fail(c, A5X_E_CAPACITY, "output needs %llu bytes, buffer has %llu", (unsigned long long)(R.b1 - R.b0),
                (unsigned long long)out_cap);
  if (J.mode != A5X_MODE_DEFAULT) {
    A5xModeLaunch M = mode_launch(c, J.w, J.wo, J.nw, J.mode, J.mn, J.mx, J.B.rfast);
    M.cand_off = J.B.cand_off;
    M.item_begin = R.i0;
    M.item_end = R.i1;
    M.cand_begin = R.cb;
    M.cand_end = R.ce;
    M.out = d_out;
    M.out_base = R.b0;
    M.out_cap = out_cap;
    if (!J.B.rfast) {
      HIPCHK(c, a5x_launch_mode_items(M, 1, J.st));
      return A5X_OK;
    }
    // -r FAST words: k_expand_fast on the job stream, the mode engine's items (disjoint
    // output bytes) on the side stream, joined before the range completes
    if (!c->sstream) HIPCHK(c, hipStreamCreateWithFlags(&c->sstream, hipStreamNonBlocking));
    if (!c->ev_fork) HIPCHK(c, hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
    if (!c->ev_join) HIPCHK(c, hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->ev_fork, J.st));
    HIPCHK(c, hipStreamWaitEvent(c->sstream, c->ev_fork, 0));
    // a few mode words among many FAST ones: a small grid filters the items beside k_expand_fast
    // instead of one workgroup per 64 items (C5 -s A/B, profiles/r05g_ab_mode_items_grid_c5.txt)
    M.grid_cap = J.B.nmode * 8 < J.nw ? 2048u : 0u;
    if (J.B.nmode) HIPCHK(c, a5x_launch_mode_items(M, 1, c->sstream));  // (every word FAST: none)
    A5xExpLaunch E = exp_launch_mode(c, J.w, J.wo, J.nw, J.mn, J.mx, J.B);
    E.cand_begin = R.cb;
    E.cand_end = R.ce;
    E.out = d_out;
    E.out_base = R.b0;
    E.out_cap = out_cap;
    HIPCHK(c, a5x_launch_expand(E, 0, J.st));
    HIPCHK(c, hipEventRecord(c->ev_join, c->sstream));
    HIPCHK(c, hipStreamWaitEvent(J.st, c->ev_join, 0));
    return A5X_OK;
  }
  const Batch& B = J.B;
  A5xExpLaunch E = exp_launch(c, J.w, J.wo, J.nw, J.mn, J.mx, B);
  E.cand_begin = R.cb;
  E.cand_end = R.ce;
  E.out = d_out;
  E.out_base = R.b0;
  E.out_cap = out_cap;
  // slow / BIG words: (word, SEG-candidate segment) items, slow from segs[0], BIG
  // from segs[sbound]; a word adds at most ceil(range / SEG) + 1 segments
  const uint64_t rng_segs = (R.ce - R.cb) / c->seg + 1;
  const uint64_t sbound = B.nslow ? B.nslow + rng_segs : 0;
  const uint64_t bbound = B.nbig ? B.nbig + rng_segs : 0;
  if (sbound + bbound > 0xffffffffull)
    return fail(c, A5X_E_CAPACITY, "call range needs more than 2^32 slow-path segments (lower A5X_CHUNK range)");
  if (B.nslow || B.nbig) {
    if ((rc = grow(c, c->segs, sbound + bbound + 1))) return rc;
    HIPCHK(c, hipMemsetAsync(c->d_scalars + 5, 0, 8, J.st));
  }
  if (B.nslow)
    HIPCHK(c, a5x_launch_segments(c->slow_list.p, c->d_scalars + 3, B.nslow, B.cand_off, R.cb, R.ce, c->seg,
                                  c->segs.p, c->d_scalars + 5, J.st));
  if (B.nbig)
    HIPCHK(c, a5x_launch_segments(c->big_list.p, c->d_scalars + 1, B.nbig, B.cand_off, R.cb, R.ce, c->seg,
                                  c->segs.p + sbound, c->d_scalars + 6, J.st));
  hipStream_t side = J.st;
  if (B.nslow || B.nbig) {
    if (!c->sstream) HIPCHK(c, hipStreamCreateWithFlags(&c->sstream, hipStreamNonBlocking));
    if (!c->ev_fork) HIPCHK(c, hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
    if (!c->ev_join) HIPCHK(c, hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->ev_fork, J.st));
    HIPCHK(c, hipStreamWaitEvent(c->sstream, c->ev_fork, 0));
    side = c->sstream;
  }
  if (B.nslow) {
    E.segs = c->segs.p; E.nsegs = c->d_scalars + 5; E.nsegs_bound = sbound;
    HIPCHK(c, a5x_launch_expand(E, 1, side));
  }
  if (B.nbig) {
    E.segs = c->segs.p + sbound; E.nsegs = c->d_scalars + 6; E.nsegs_bound = bbound;
    HIPCHK(c, a5x_launch_expand(E, 2, side));
    if (B.nglob) HIPCHK(c, a5x_launch_expand(E, 4, side));  // pass G words of the same list
  }
  HIPCHK(c, a5x_launch_expand(E, 0, J.st));
  if (side != J.st) {
    HIPCHK(c, hipEventRecord(c->ev_join, side));
    HIPCHK(c, hipStreamWaitEvent(J.st, c->ev_join, 0));
  }
  return A5X_OK;
}

int job_open(a5x_ctx* c, Job& J, const uint8_t* d_words, const uint64_t* d_woff, uint64_t nw, int mode, int mn,
             int mx, hipStream_t st) {
  J.w = d_words; J.wo = d_woff; J.nw = nw; J.mode = mode; J.mn = mn; J.mx = mx; J.st = st;
  return A5X_OK;
}

// ---------------------------------------------------------------------------
// fused digest + lookup (a5x_digest.hip)
// ---------------------------------------------------------------------------
inline uint64_t tgt_slot(const uint32_t* d, uint64_t tmask) {
  const uint64_t h = ((uint64_t)d[1] | ((uint64_t)d[2] << 32)) * 0x9E3779B97F4A7C15ull;  // == probe()
  return (h >> 20) & tmask;
}

A5xDigLaunch dig_launch(a5x_ctx* c) {
  A5xDigLaunch D;
  memset(&D, 0, sizeof D);
  D.algo = c->t_algo < 0 ? A5X_ALGO_MD5 : c->t_algo;
  D.bitmap = c->t_bitmap.p;
  D.bm_mask = c->t_bm_log2 >= 32 ? 0xffffffffu : (uint32_t)((1ull << c->t_bm_log2) - 1);
  D.table = c->t_table.p; D.tmask = c->t_tmask; D.has_zero_target = c->t_has_zero;
  D.err = c->d_scalars + 2;
  return D;
}

uint32_t dig_grid(a5x_ctx* c) { return (uint32_t)std::max(1, c->cus) * 8u; }

// per-2KiB-block line starts and their exclusive scan (blk_pre, nblk+1 entries)
int dig_block_prefix(a5x_ctx* c, A5xDigLaunch& D, hipStream_t st, uint64_t* total_lines) {
  int rc;
  const uint64_t nblk = a5x_digest_blocks(D.nbytes, D.algo);
  if ((rc = grow(c, c->dg_blk_cnt, nblk + 1)) || (rc = grow(c, c->dg_blk_pre, nblk + 1)) ||
      (rc = grow(c, c->scan_tmp, a5x_scan_tmp_elems(nblk + 1) + 16)))
    return rc;
  D.blk_cnt = c->dg_blk_cnt.p;
  HIPCHK(c, a5x_launch_digest_stream(D, 1, dig_grid(c), st));
  HIPCHK(c, a5x_launch_scan(c->dg_blk_cnt.p, c->dg_blk_cnt.p, nblk, c->dg_blk_pre.p, c->dg_blk_pre.p, c->scan_tmp.p,
                            c->d_scalars + 2, st));
  D.blk_pre = c->dg_blk_pre.p;
  if (total_lines) {
    HIPCHK(c, hipMemcpyAsync(c->h_totals + 2, c->dg_blk_pre.p + nblk, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    *total_lines = c->h_totals[2];
  }
  return A5X_OK;
}

static_assert(sizeof(a5x_hit) == sizeof(A5xHitRaw), "resolved device hits are copied out as a5x_hit");

// a5x_expand_digest_device.  allow_fused: default-mode batches take the fused kernel
// (the hybrid's sub-batch of non-FAST words passes false: those words are exactly the
// ones the fused kernel skips).
// The item range [*i0, *i1) of the -r / -s engines holding candidates [cb, ce) (ce <= the
// batch's count, cb < ce): the words of cb and ce - 1 from k_word_of, their first items.
int mode_item_bounds(a5x_ctx* c, const Job& J, uint64_t cb, uint64_t ce, uint64_t* i0, uint64_t* i1) {
  int rc;
  if ((rc = grow(c, c->loc_q, 2)) || (rc = grow(c, c->loc_r, 4))) return rc;
  const uint64_t q[2] = {cb, ce - 1};
  HIPCHK(c, hipMemcpyAsync(c->loc_q.p, q, 16, hipMemcpyHostToDevice, J.st));
  HIPCHK(c, a5x_launch_word_of(J.B.cand_off, J.nw, c->loc_q.p, 2, c->loc_r.p, c->loc_r.p + 2, J.st));
  uint64_t wc[4], so[2];
  HIPCHK(c, hipMemcpyAsync(wc, c->loc_r.p, 32, hipMemcpyDeviceToHost, J.st));
  HIPCHK(c, hipStreamSynchronize(J.st));
  for (int k = 0; k < 2; k++) {
    if (wc[k] >= J.nw) return fail(c, A5X_E_ARG, "candidate %llu past the batch", (unsigned long long)q[k]);
    HIPCHK(c, hipMemcpyAsync(&so[k], c->m_seg_off.p + wc[k], 8, hipMemcpyDeviceToHost, J.st));
  }
  HIPCHK(c, hipStreamSynchronize(J.st));
  *i0 = so[0] + wc[2] / c->mseg;
  *i1 = so[1] + wc[3] / c->mseg + 1;
  return A5X_OK;
}

// Fused (or two-pass) expansion + digest + lookup of the batch's candidates [rb, re)
// (clipped to the batch; [0, ~0) = all): hits as (word, candidate in word).
int expand_digest(a5x_ctx* c, const uint8_t* d_words, const uint64_t* d_woff, uint64_t nw, int mode, int mn, int mx,
                  uint64_t rb, uint64_t re, uint64_t scratch_bytes, a5x_hit* hits, uint64_t hit_cap,
                  uint64_t* n_hits, a5x_stats* stats, hipStream_t st, bool allow_fused, uint64_t trim = 0) {
  int rc;
  Job J;
  job_open(c, J, d_words, d_woff, nw, mode, mn, mx, st);
  J.lengths = mode == A5X_MODE_DEFAULT || !allow_fused;  // the fused -r / -s digest needs no layout
  if ((rc = grow(c, c->dg_cand_off, nw + 1)) || (rc = grow(c, c->dg_byte_off, nw + 1))) return rc;
  if ((rc = job_prepare(c, J, c->dg_cand_off.p, c->dg_byte_off.p, true))) return rc;
  const uint64_t tc_all = J.B.total_cands, tb = J.B.total_bytes;
  re = std::min(re, tc_all - std::min(trim, tc_all));  // (trim: candidates dropped at the end)
  rb = std::min(rb, re);
  const bool whole = rb == 0 && re == tc_all;
  const uint64_t tc = re - rb;  // the candidates this call digests
  // Fused path (default mode): k_expand_fast_md5 / k_expand_fast_ntlm hash each FAST
  // word's candidates in the LDS ring where they are built -- no HBM scratch, no second
  // pass, hits already (word, candidate).  The other candidate-bearing words (slow / BIG
  // / pass G) are gathered into a sub-batch for the two-pass path (hybrid).  Modes
  // -r / -s / -s -r: the two-pass range loop below.
  if (mode != A5X_MODE_DEFAULT && allow_fused) {
    // -r / -s / -s -r: every item's candidates hashed where the engine builds them
    // (positional ring or byte-builder buffer), hits as (word, candidate) directly
    uint64_t dev_hits = std::max<uint64_t>(1024, std::min<uint64_t>(hit_cap, 1u << 20));
    if ((rc = grow(c, c->dg_hits, dev_hits))) return rc;
    uint64_t nh = 0;
    float ms = 0;
    uint64_t it0 = 0, it1 = c->m_items;  // the items holding [rb, re)
    if (!whole && tc && (rc = mode_item_bounds(c, J, rb, re, &it0, &it1))) return rc;
    for (;;) {
      A5xModeLaunch M = mode_launch(c, J.w, J.wo, J.nw, J.mode, J.mn, J.mx, J.B.rfast);
      const A5xDigLaunch D = dig_launch(c);
      M.cand_off = J.B.cand_off;
      M.item_begin = it0;
      M.item_end = tc ? it1 : it0;
      M.cand_begin = rb;
      M.cand_end = re;
      M.dg_algo = c->t_algo;
      M.dg_bitmap = D.bitmap; M.dg_bm_mask = D.bm_mask; M.dg_has_zero = D.has_zero_target;
      M.dg_table = D.table; M.dg_tmask = D.tmask;
      M.dg_hits = c->dg_hits.p; M.dg_hit_cap = (uint32_t)dev_hits; M.dg_nhits = c->d_scalars + 8;
      HIPCHK(c, hipMemsetAsync(c->d_scalars + 8, 0, 4, J.st));
      HIPCHK(c, hipEventRecord(c->ev[1], J.st));
      M.grid_cap = J.B.nmode * 8 < J.nw ? 2048u : 0u;  // (as in job_launch)
      if (J.B.nmode && tc) HIPCHK(c, a5x_launch_mode_items(M, 2, J.st));
      if (J.B.rfast && tc) {  // -r FAST words: hashed in k_expand_fast_md5 / _ntlm's ring
        A5xExpLaunch E = exp_launch_mode(c, J.w, J.wo, J.nw, J.mn, J.mx, J.B);
        E.cand_begin = rb;
        E.cand_end = re;
        E.dg_bitmap = D.bitmap; E.dg_bm_mask = D.bm_mask; E.dg_has_zero = D.has_zero_target;
        E.dg_table = D.table; E.dg_tmask = D.tmask;
        E.dg_hits = c->dg_hits.p; E.dg_hit_cap = (uint32_t)dev_hits; E.dg_nhits = c->d_scalars + 8;
        HIPCHK(c, a5x_launch_expand(E, c->t_algo == A5X_ALGO_MD5 ? 3 : 5, J.st));
      }
      HIPCHK(c, hipEventRecord(c->ev[2], J.st));
      HIPCHK(c, hipMemcpyAsync(c->h_scalars, c->d_scalars, 64, hipMemcpyDeviceToHost, J.st));
      HIPCHK(c, hipStreamSynchronize(J.st));
      HIPCHK(c, hipEventElapsedTime(&ms, c->ev[1], c->ev[2]));
      if ((rc = decode_dev_err(c, c->h_scalars[2]))) return rc;
      nh = c->h_scalars[8];
      if (nh <= dev_hits || hit_cap <= dev_hits) break;
      dev_hits = std::min<uint64_t>(nh, hit_cap);  // run again with room for every hit the caller takes
      if ((rc = grow(c, c->dg_hits, dev_hits))) return rc;
    }
    const uint64_t take = std::min(std::min(nh, dev_hits), hit_cap);
    if (take) {
      HIPCHK(c, hipMemcpyAsync(hits, c->dg_hits.p, take * sizeof(a5x_hit), hipMemcpyDeviceToHost, J.st));
      HIPCHK(c, hipStreamSynchronize(J.st));
    }
    float a = 0;
    HIPCHK(c, hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
    a5x_stats total;
    memset(&total, 0, sizeof total);
    total.words = nw;
    total.candidates = tc;
    total.expand_launches = 1;
    total.ms_keyspace = a;
    total.ms_expand = ms;  // build + digest + lookup, fused
    total.ms_total = a + ms;
    if (n_hits) *n_hits = nh;
    if (stats) *stats = total;
    if (nh > hit_cap)
      return fail(c, A5X_E_CAPACITY, "%llu hits, buffer has %llu", (unsigned long long)nh, (unsigned long long)hit_cap);
    return A5X_OK;
  }
  const bool fused = mode == A5X_MODE_DEFAULT && tc > 0 && allow_fused;
  const bool hybrid = fused && (J.B.nslow || J.B.nbig || J.B.nglob);
  if (fused) {
    uint64_t dev_hits = std::max<uint64_t>(1024, std::min<uint64_t>(hit_cap, 1u << 20));
    if ((rc = grow(c, c->dg_hits, dev_hits))) return rc;
    uint64_t nh = 0;
    float ms = 0;
    for (;;) {
      A5xExpLaunch E = exp_launch(c, J.w, J.wo, J.nw, J.mn, J.mx, J.B);
      const A5xDigLaunch D = dig_launch(c);
      E.cand_begin = rb;
      E.cand_end = re;
      E.dg_bitmap = D.bitmap; E.dg_bm_mask = D.bm_mask; E.dg_has_zero = D.has_zero_target;
      E.dg_table = D.table; E.dg_tmask = D.tmask;
      E.dg_hits = c->dg_hits.p; E.dg_hit_cap = (uint32_t)dev_hits; E.dg_nhits = c->d_scalars + 8;
      HIPCHK(c, hipMemsetAsync(c->d_scalars + 8, 0, 4, J.st));
      HIPCHK(c, hipEventRecord(c->ev[1], J.st));
      HIPCHK(c, a5x_launch_expand(E, c->t_algo == A5X_ALGO_MD5 ? 3 : 5, J.st));
      HIPCHK(c, hipEventRecord(c->ev[2], J.st));
      HIPCHK(c, hipMemcpyAsync(c->h_scalars, c->d_scalars, 64, hipMemcpyDeviceToHost, J.st));
      HIPCHK(c, hipStreamSynchronize(J.st));
      HIPCHK(c, hipEventElapsedTime(&ms, c->ev[1], c->ev[2]));
      if ((rc = decode_dev_err(c, c->h_scalars[2]))) return rc;
      nh = c->h_scalars[8];
      if (nh <= dev_hits || hit_cap <= dev_hits) break;
      dev_hits = std::min<uint64_t>(nh, hit_cap);  // run again with room for every hit the caller takes
      if ((rc = grow(c, c->dg_hits, dev_hits))) return rc;
    }
    uint64_t take = std::min(std::min(nh, dev_hits), hit_cap);
    if (take) {
      HIPCHK(c, hipMemcpyAsync(hits, c->dg_hits.p, take * sizeof(a5x_hit), hipMemcpyDeviceToHost, J.st));
      HIPCHK(c, hipStreamSynchronize(J.st));
    }
    float a = 0;  // this batch's keyspace (before the sub-batch reuses the events)
    HIPCHK(c, hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
    float ms_sub = 0;
    if (hybrid) {
      // The words the fused kernel skipped, in batch order, as a compact sub-batch in
      // the context's hybrid buffers (sized with grow(): no per-call allocation).
      // Host memory touched with device-produced values: idx[] (sized by the device count
      // m, itself bounded by nw) and the caller's hits[take, take + got) with got <= room.
      if ((rc = grow(c, c->hy_list, std::max<uint64_t>(1, nw)))) return rc;
      HIPCHK(c, hipMemsetAsync(c->d_scalars + 9, 0, 4, J.st));
      HIPCHK(c, a5x_launch_nonfast_list(c->flags.p, J.B.cand_off, nw, rb, re, c->hy_list.p, c->d_scalars + 9, J.st));
      HIPCHK(c, hipMemcpyAsync(c->h_scalars + 9, c->d_scalars + 9, 4, hipMemcpyDeviceToHost, J.st));
      HIPCHK(c, hipStreamSynchronize(J.st));
      const uint32_t m = c->h_scalars[9];
      if (m > nw) return fail(c, A5X_E_HIP, "non-FAST word list of %u words in a batch of %llu", m, (unsigned long long)nw);
      std::vector<uint32_t> idx(m);
      std::vector<uint64_t> off((size_t)m + 1, 0);
      if ((rc = grow(c, c->hy_lens, (size_t)m + 1)) || (rc = grow(c, c->hy_off, (size_t)m + 1))) return rc;
      if (m) {
        HIPCHK(c, hipMemcpyAsync(idx.data(), c->hy_list.p, (size_t)m * 4, hipMemcpyDeviceToHost, J.st));
        HIPCHK(c, hipStreamSynchronize(J.st));
        std::sort(idx.begin(), idx.end());
        HIPCHK(c, hipMemcpyAsync(c->hy_list.p, idx.data(), (size_t)m * 4, hipMemcpyHostToDevice, J.st));
        HIPCHK(c, a5x_launch_gather_words(J.w, J.wo, c->hy_list.p, m, c->hy_lens.p, nullptr, nullptr, J.st));
        HIPCHK(c, hipMemcpyAsync(off.data() + 1, c->hy_lens.p, (size_t)m * 8, hipMemcpyDeviceToHost, J.st));
        HIPCHK(c, hipStreamSynchronize(J.st));
        for (uint32_t k = 0; k < m; k++) off[k + 1] += off[k];
      }
      if ((rc = grow(c, c->hy_words, off[m] + 16))) return rc;
      HIPCHK(c, hipMemcpyAsync(c->hy_off.p, off.data(), ((size_t)m + 1) * 8, hipMemcpyHostToDevice, J.st));
      HIPCHK(c, hipMemsetAsync(c->hy_words.p, 0, off[m] + 16, J.st));
      HIPCHK(c, a5x_launch_gather_words(J.w, J.wo, c->hy_list.p, m, nullptr, c->hy_off.p, c->hy_words.p, J.st));
      // their candidates through the two-pass path; hit word indices mapped back to the batch.
      // A word cut by [rb, re) (the first / last listed): only its part inside the range --
      // the sub-batch range drops the candidates before rb and after re.
      uint64_t sb = 0, se_cut = 0;
      if (m && !whole) {
        uint64_t c0 = 0, c1 = 0;
        HIPCHK(c, hipMemcpyAsync(&c0, J.B.cand_off + idx[0], 8, hipMemcpyDeviceToHost, J.st));
        HIPCHK(c, hipMemcpyAsync(&c1, J.B.cand_off + idx[m - 1] + 1, 8, hipMemcpyDeviceToHost, J.st));
        HIPCHK(c, hipStreamSynchronize(J.st));
        sb = rb > c0 ? rb - c0 : 0;
        se_cut = c1 > re ? c1 - re : 0;
      }
      const uint64_t room = hit_cap > take ? hit_cap - take : 0;
      uint64_t nh2 = 0;
      a5x_stats st2;
      memset(&st2, 0, sizeof st2);
      rc = expand_digest(c, c->hy_words.p, c->hy_off.p, m, mode, mn, mx, sb, ~0ull, scratch_bytes,
                         room ? hits + take : nullptr, room, &nh2, &st2, J.st, false, se_cut);
      if (rc && rc != A5X_E_CAPACITY) return rc;
      const uint64_t got = std::min(nh2, room);
      for (uint64_t i = take; i < take + got; i++) {
        if (hits[i].word >= m)
          return fail(c, A5X_E_HIP, "sub-batch hit word %llu of %u", (unsigned long long)hits[i].word, m);
        hits[i].word = idx[hits[i].word];
      }
      take += got;
      nh += nh2;
      ms_sub = st2.ms_total;
    }
    a5x_stats total;
    memset(&total, 0, sizeof total);
    total.words = nw;
    total.candidates = tc;
    total.bytes = tb;
    total.expand_launches = 1;
    total.ms_keyspace = a;
    total.ms_expand = ms + ms_sub;  // expansion + digest + lookup: fused (+ the two-pass sub-batch)
    total.ms_total = a + ms + ms_sub;
    if (n_hits) *n_hits = nh;
    if (stats) *stats = total;
    if (nh > hit_cap)
      return fail(c, A5X_E_CAPACITY, "%llu hits, buffer has %llu", (unsigned long long)nh,
                  (unsigned long long)hit_cap);
    return A5X_OK;
  }
  uint64_t cap = scratch_bytes ? scratch_bytes : ((uint64_t)2 << 30);
  cap = std::max<uint64_t>(4096, std::min<uint64_t>(cap, tb + 64));
  std::vector<Range> ranges;
  if ((rc = plan_ranges(c, J, cap, ranges, rb, re))) return rc;
  if ((rc = grow(c, c->dg_scratch, cap + 64))) return rc;
  uint64_t dev_hits = std::max<uint64_t>(1024, std::min<uint64_t>(hit_cap, 1u << 20));
  if ((rc = grow(c, c->dg_hits, dev_hits))) return rc;
  a5x_stats total;
  memset(&total, 0, sizeof total);
  total.words = nw;
  total.candidates = tc;
  total.bytes = tb;
  uint64_t found = 0, copied = 0;
  float ms_exp = 0, ms_dig = 0, ms_ks = 0;
  HIPCHK(c, hipEventRecord(c->ev[3], J.st));  // the keyspace (and the range plan) ends here
  HIPCHK(c, hipEventSynchronize(c->ev[3]));
  HIPCHK(c, hipEventElapsedTime(&ms_ks, c->ev[0], c->ev[3]));
  for (const Range& R : ranges) {
    HIPCHK(c, hipEventRecord(c->ev[1], J.st));
    if ((rc = job_launch(c, J, R, c->dg_scratch.p, cap))) return rc;
    HIPCHK(c, hipEventRecord(c->ev[2], J.st));
    A5xDigLaunch D = dig_launch(c);
    D.out = c->dg_scratch.p;
    D.nbytes = R.b1 - R.b0;
    const uint64_t nblk = a5x_digest_blocks(D.nbytes, D.algo);
    if ((rc = grow(c, c->dg_blk_cnt, nblk + 1)) || (rc = grow(c, c->dg_blk_pre, nblk + 1)) ||
        (rc = grow(c, c->scan_tmp, a5x_scan_tmp_elems(nblk + 1) + 16)))
      return rc;
    D.blk_cnt = c->dg_blk_cnt.p;
    uint64_t nh = 0;
    {
      float me = 0;  // the range's expansion, once (a retry below re-runs only the digest)
      HIPCHK(c, hipEventSynchronize(c->ev[2]));
      HIPCHK(c, hipEventElapsedTime(&me, c->ev[1], c->ev[2]));
      ms_exp += me;
    }
    for (;;) {  // a range with more hits than the device buffer is digested again with room for all
      D.hits = c->dg_hits.p;
      D.hit_cap = (uint32_t)dev_hits;
      D.nhits = c->d_scalars + 8;
      HIPCHK(c, hipMemsetAsync(c->d_scalars + 8, 0, 4, J.st));
      HIPCHK(c, hipEventRecord(c->dev_ev[0], J.st));
      HIPCHK(c, a5x_launch_digest_stream(D, 0, dig_grid(c), J.st));
      HIPCHK(c, hipEventRecord(c->dev_ev[1], J.st));
      HIPCHK(c, hipMemcpyAsync(c->h_scalars, c->d_scalars, 64, hipMemcpyDeviceToHost, J.st));
      HIPCHK(c, hipStreamSynchronize(J.st));
      float md = 0;
      HIPCHK(c, hipEventElapsedTime(&md, c->dev_ev[0], c->dev_ev[1]));
      ms_dig += md;
      const uint32_t e = c->h_scalars[2] & ~(1u << 10);
      if ((rc = decode_dev_err(c, e))) return rc;
      nh = c->h_scalars[8];
      if (nh <= dev_hits || copied >= hit_cap) break;
      dev_hits = nh;  // grow and run this range's digest again (its candidates are still in scratch)
      if ((rc = grow(c, c->dg_hits, dev_hits))) return rc;
      HIPCHK(c, hipMemsetAsync(c->d_scalars + 2, 0, 4, J.st));
    }
    if (nh) {
      const uint64_t got = std::min<uint64_t>(nh, dev_hits);
      HIPCHK(c, a5x_launch_scan(c->dg_blk_cnt.p, c->dg_blk_cnt.p, nblk, c->dg_blk_pre.p, c->dg_blk_pre.p,
                                c->scan_tmp.p, c->d_scalars + 2, J.st));
      HIPCHK(c, a5x_launch_hits_resolve(c->dg_hits.p, (uint32_t)got, c->dg_blk_pre.p, R.cb, c->dg_cand_off.p, nw,
                                        J.st));
      const uint64_t take = std::min(hit_cap - std::min(hit_cap, copied), got);
      if (take)
        HIPCHK(c, hipMemcpyAsync(hits + copied, c->dg_hits.p, take * sizeof(a5x_hit), hipMemcpyDeviceToHost, J.st));
      HIPCHK(c, hipStreamSynchronize(J.st));
      copied += take;
      found += nh;
    }
    total.expand_launches += 1;
  }
  total.ms_keyspace = ms_ks;
  total.ms_expand = ms_exp;
  total.ms_total = total.ms_keyspace + ms_exp + ms_dig;
  total.words_slow = J.B.nslow;
  total.words_pass_b = J.B.nbig;
  if (n_hits) *n_hits = found;
  if (stats) *stats = total;
  if (found > hit_cap)
    return fail(c, A5X_E_CAPACITY, "%llu hits, buffer has %llu", (unsigned long long)found,
                (unsigned long long)hit_cap);
  return A5X_OK;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int a5x_abi_version(void) { return A5X_ABI_VERSION; }

// Why the calling thread's last a5x_create failed (no context exists to carry
// a5x_last_error): the failing HIP call and hipGetErrorString, or the argument problem.
static thread_local std::string g_create_err;

static int create_fail(int rc, const char* call, hipError_t e, int device) {
  char buf[256];
  if (e != hipSuccess)
    snprintf(buf, sizeof buf, "a5x_create(device=%d): %s failed: %s (hipError_t %d)", device, call,
             hipGetErrorString(e), (int)e);
  else
    snprintf(buf, sizeof buf, "a5x_create(device=%d): %s", device, call);
  g_create_err = buf;
  return rc;
}

int a5x_create(int device, a5x_ctx** out) {
  g_create_err.clear();
  if (!out) return create_fail(A5X_E_ARG, "null output pointer", hipSuccess, device);
  *out = nullptr;
  if (device == -1) {  // host-only context: tables, splitting, export (no GPU needed)
    a5x_ctx* c = new a5x_ctx();
    c->device = -1;
    *out = c;
    return A5X_OK;
  }
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) return create_fail(A5X_E_HIP, "hipGetDeviceCount", e, device);
  if (n <= 0) return create_fail(A5X_E_HIP, "hipGetDeviceCount found no device", hipSuccess, device);
  if (device < 0 || device >= n) {
    char msg[96];
    snprintf(msg, sizeof msg, "device out of range (%d visible)", n);
    return create_fail(A5X_E_ARG, msg, hipSuccess, device);
  }
  a5x_ctx* c = new a5x_ctx();
  c->device = device;
  if ((e = hipSetDevice(device)) != hipSuccess) {
    delete c;
    return create_fail(A5X_E_HIP, "hipSetDevice", e, device);
  }
  if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) {
    delete c;
    return create_fail(A5X_E_HIP, "hipStreamCreateWithFlags", e, device);
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
    c->devname = std::string(prop.name) + " (" + prop.gcnArchName + ")";
    c->cus = prop.multiProcessorCount;
  }
  if (c->cus <= 0) c->cus = 256;
  const char* what = nullptr;
  if ((e = hipMalloc((void**)&c->d_scalars, 256)) != hipSuccess) what = "hipMalloc";
  else if ((e = hipHostMalloc((void**)&c->h_scalars, 256, 0)) != hipSuccess) what = "hipHostMalloc";
  else if ((e = hipHostMalloc((void**)&c->h_totals, 64, 0)) != hipSuccess) what = "hipHostMalloc";
  else if ((e = a5x_set_kernel_attrs()) != hipSuccess) what = "hipFuncSetAttribute";
  for (int i = 0; i < 4 && !what; i++)
    if ((e = hipEventCreate(&c->ev[i])) != hipSuccess) what = "hipEventCreate";
  for (int i = 0; i < 2 && !what; i++)
    if ((e = hipEventCreate(&c->dev_ev[i])) != hipSuccess) what = "hipEventCreate";
  if (what) {
    a5x_destroy(c);
    return create_fail(A5X_E_HIP, what, e, device);
  }
  if (const char* e = getenv("A5X_CHUNK")) c->chunk = std::max<uint64_t>(64, strtoull(e, nullptr, 10));
  // (< 2^24: k_keyspace_vsub packs a sub-word count <= mseg into 24 bits)
  if (const char* e = getenv("A5X_MSEG")) c->mseg = std::min<uint64_t>((1u << 24) - 1, std::max<uint64_t>(1, strtoull(e, nullptr, 10)));
  if (const char* e = getenv("A5X_SEG")) c->seg = std::max<uint64_t>(64, strtoull(e, nullptr, 10));
  // (tuning knobs; a5x_launch_expand clamps each launch to the kernel's compiled launch bound)
  if (const char* e = getenv("A5X_WAVES")) c->waves_per_block = std::max(1u, std::min(16u, (unsigned)atoi(e)));
  if (const char* e = getenv("A5X_FAST_WAVES")) c->waves_per_block_fast = std::max(1u, std::min(16u, (unsigned)atoi(e)));
  *out = c;
  return A5X_OK;
}

void a5x_destroy(a5x_ctx* c) {
  if (!c) return;
  if (c->device < 0) { delete c; return; }
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  release(c->count); release(c->bytes); release(c->cand_off); release(c->byte_off); release(c->scan_tmp);
  release(c->locate); release(c->flags); release(c->defer); release(c->chunk_w0); release(c->slow_list); release(c->big_list);
  release(c->segs);
  release(c->m_nseg); release(c->m_seg_off); release(c->m_seg_bytes); release(c->m_item_fl); release(c->m_seg_boff); release(c->m_tmp);
  release(c->m_item_w);
  release(c->t_bitmap); release(c->t_table); release(c->dg_scratch); release(c->dg_blk_cnt); release(c->dg_blk_pre);
  release(c->dg_cand_off); release(c->dg_byte_off); release(c->dg_hits);
  release(c->hy_list); release(c->hy_lens); release(c->hy_off); release(c->hy_words);
  for (auto& e : c->dev_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->d_mtab) (void)hipFree(c->d_mtab);
  release(c->s_words); release(c->s_out[0]); release(c->s_out[1]); release(c->s_woff);
  release(c->loc_q); release(c->loc_r);
  for (auto& e : c->ev_exp)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->ev_cpy)
    if (e) (void)hipEventDestroy(e);
  if (c->cstream) (void)hipStreamDestroy(c->cstream);
  release(c->glob);
  release(c->m_vl); release(c->vn); release(c->vrsz); release(c->vpre); release(c->vrpre); release(c->vrec);
  release(c->vrec2); release(c->vcand_off); release(c->vbyte_off); release(c->vflags); release(c->vroff);
  release(c->vmap); release(c->vobase); release(c->vocc);
  if (c->mgscr) (void)hipFree(c->mgscr);
  if (c->gscr) (void)hipFree(c->gscr);
  if (c->sstream) (void)hipStreamSynchronize(c->sstream);
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  if (c->sstream) (void)hipStreamDestroy(c->sstream);
  if (c->d_table) (void)hipFree(c->d_table);
  if (c->d_scalars) (void)hipFree(c->d_scalars);
  if (c->h_scalars) (void)hipHostFree(c->h_scalars);
  if (c->h_totals) (void)hipHostFree(c->h_totals);
  for (auto& h : c->h_out)
    if (h) (void)hipHostFree(h);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* a5x_last_error(const a5x_ctx* c) { return c ? c->err.c_str() : "null context"; }

const char* a5x_create_error(void) { return g_create_err.c_str(); }

int a5x_device_info(a5x_ctx* c, char* name, size_t cap, int* cu_count) {
  if (!c) return A5X_E_ARG;
  if (name && cap) {
    strncpy(name, c->devname.c_str(), cap - 1);
    name[cap - 1] = 0;
  }
  if (cu_count) *cu_count = c->cus;
  return A5X_OK;
}

int a5x_load_table_file(a5x_ctx* c, const char* path) {
  if (!c || !path) return A5X_E_ARG;
  FILE* f = fopen(path, "rb");
  if (!f) return fail(c, A5X_E_IO, "open %s: %s", path, strerror(errno));
  std::vector<uint8_t> d;
  uint8_t buf[65536];
  size_t r;
  while ((r = fread(buf, 1, sizeof buf, f)) > 0) d.insert(d.end(), buf, buf + r);
  const bool err = ferror(f);
  fclose(f);
  if (err) return fail(c, A5X_E_IO, "read %s failed", path);
  return a5x_parse_table(c, d.data(), d.size());
}

int a5x_parse_table(a5x_ctx* c, const uint8_t* data, size_t len) {
  if (!c || (!data && len)) return A5X_E_ARG;
  Table t = c->table;
  int rc = parse_table_into(c, t, data, len);
  if (rc) return rc;
  c->table = std::move(t);
  c->table_dirty = true;
  c->mtable_dirty = true;
  return A5X_OK;
}

int a5x_set_table(a5x_ctx* c, const uint8_t* kb, const uint64_t* koff, uint32_t nk, const uint8_t* vb,
                  const uint64_t* voff, const uint32_t* vkey, uint32_t nv) {
  if (!c || (nk && !koff) || (nv && (!voff || !vkey))) return A5X_E_ARG;
  Table t;
  for (uint32_t i = 0; i < nk; i++) {
    if (koff[i + 1] < koff[i]) return fail(c, A5X_E_ARG, "key offsets not monotone");
    std::string k((const char*)kb + koff[i], (size_t)(koff[i + 1] - koff[i]));
    if (t.index.count(k)) return fail(c, A5X_E_ARG, "duplicate key %u", i);
    t.index.emplace(k, (uint32_t)t.keys.size());
    t.keys.push_back(k);
    t.vals.emplace_back();
  }
  for (uint32_t j = 0; j < nv; j++) {
    if (vkey[j] >= nk || voff[j + 1] < voff[j]) return fail(c, A5X_E_ARG, "bad value %u", j);
    t.vals[vkey[j]].emplace_back((const char*)vb + voff[j], (size_t)(voff[j + 1] - voff[j]));
  }
  c->table = std::move(t);
  c->table_dirty = true;
  c->mtable_dirty = true;
  return A5X_OK;
}

int a5x_clear_table(a5x_ctx* c) {
  if (!c) return A5X_E_ARG;
  c->table.clear();
  c->table_dirty = true;
  c->mtable_dirty = true;
  return A5X_OK;
}

int a5x_table_export(const a5x_ctx* c, uint32_t* n_keys, uint32_t* n_vals, uint64_t* key_bytes, uint64_t* val_bytes,
                     uint8_t* ko, uint64_t* koff, uint8_t* vo, uint64_t* voff, uint32_t* vkey) {
  if (!c) return A5X_E_ARG;
  const Table& t = c->table;
  uint64_t kbt = 0, vbt = 0, nv = 0;
  if (koff) koff[0] = 0;
  if (voff) voff[0] = 0;
  for (uint32_t i = 0; i < t.keys.size(); i++) {
    if (ko) memcpy(ko + kbt, t.keys[i].data(), t.keys[i].size());
    kbt += t.keys[i].size();
    if (koff) koff[i + 1] = kbt;
    for (auto& v : t.vals[i]) {
      if (vo) memcpy(vo + vbt, v.data(), v.size());
      vbt += v.size();
      if (vkey) vkey[nv] = i;
      nv++;
      if (voff) voff[nv] = vbt;
    }
  }
  if (n_keys) *n_keys = (uint32_t)t.keys.size();
  if (n_vals) *n_vals = (uint32_t)nv;
  if (key_bytes) *key_bytes = kbt;
  if (val_bytes) *val_bytes = vbt;
  return A5X_OK;
}

int a5x_split_words(const uint8_t* data, size_t len, uint8_t* words_out, uint64_t* off_out, uint64_t off_cap,
                    uint64_t* n_words) {
  if ((!data && len) || !n_words) return A5X_E_ARG;
  size_t pos = 0, wb = 0;
  uint64_t n = 0;
  const uint8_t* line;
  size_t l;
  if (off_out && off_cap) off_out[0] = 0;
  while (a5x::gosem::scan_line(data, len, &pos, &line, &l) == 1) {  // ErrTooLong: silently stop
    if (words_out) {
      if (!off_out || n + 1 >= off_cap) return A5X_E_ARG;
      memcpy(words_out + wb, line, l);
    }
    wb += l;
    n++;
    if (words_out) off_out[n] = wb;
  }
  *n_words = n;
  return A5X_OK;
}

int a5x_keyspace_device(a5x_ctx* c, const uint8_t* d_words, const uint64_t* d_woff, uint64_t nw, int mode, int mn,
                        int mx, uint64_t* d_cand_off, uint64_t* d_byte_off, uint64_t* tc, uint64_t* tb,
                        void* stream) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || (nw && (!d_words || !d_woff))) return A5X_E_ARG;
  int rc;
  if ((rc = check_mode(c, mode))) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  Batch B;
  if (mode != A5X_MODE_DEFAULT)
    rc = run_keyspace_mode(c, d_words, d_woff, nw, mode, mn, mx, d_cand_off, d_byte_off, st, &B, false);
  else
    rc = run_keyspace(c, d_words, d_woff, nw, mn, mx, d_cand_off, d_byte_off, st, &B, false);
  if (rc) return rc;
  if (tc) *tc = B.total_cands;
  if (tb) *tb = B.total_bytes;
  return A5X_OK;
}

int a5x_expand_device(a5x_ctx* c, const uint8_t* d_words, const uint64_t* d_woff, uint64_t nw, int mode, int mn,
                      int mx, uint64_t cand_begin, uint64_t cand_end, uint8_t* d_out, uint64_t out_cap,
                      uint64_t* d_cand_off, uint64_t* d_byte_off, a5x_stats* stats, void* stream) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || (nw && (!d_words || !d_woff))) return A5X_E_ARG;
  int rc;
  if ((rc = check_mode(c, mode))) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  Job J;
  job_open(c, J, d_words, d_woff, nw, mode, mn, mx, stream ? (hipStream_t)stream : c->stream);
  if ((rc = job_prepare(c, J, d_cand_off, d_byte_off, true))) return rc;
  const Batch& B = J.B;
  const uint64_t cb = std::min(cand_begin, B.total_cands);
  const uint64_t ce = std::min(cand_end, B.total_cands);
  if (stats) {
    memset(stats, 0, sizeof *stats);
    stats->words = nw;
  }
  if (ce <= cb) return A5X_OK;
  Range R{cb, ce, 0, B.total_bytes, 0, mode != A5X_MODE_DEFAULT ? c->m_items : 0};
  if (cb > 0 || ce < B.total_cands) {
    std::vector<uint64_t> res;
    if ((rc = job_locate(c, J, {cb, ce}, res))) return rc;
    R = range_of(J, cb, ce, &res[0], &res[3]);
  }
  if (stats) {
    stats->candidates = ce - cb;
    stats->bytes = R.b1 - R.b0;
  }
  HIPCHK(c, hipEventRecord(c->ev[1], J.st));
  if ((rc = job_launch(c, J, R, d_out, out_cap))) return rc;
  HIPCHK(c, hipEventRecord(c->ev[2], J.st));
  if ((rc = job_check(c, J))) return rc;
  if (stats) {
    float a = 0, b = 0, t = 0;
    HIPCHK(c, hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
    HIPCHK(c, hipEventElapsedTime(&b, c->ev[1], c->ev[2]));
    HIPCHK(c, hipEventElapsedTime(&t, c->ev[0], c->ev[2]));
    stats->ms_keyspace = a;
    stats->ms_expand = b;
    stats->ms_total = t;
    stats->words_pass_b = B.nbig;
    stats->expand_launches = mode != A5X_MODE_DEFAULT ? 1 : 1 + (B.nslow ? 1 : 0) + (B.nbig ? 1 : 0);
    stats->words_slow = B.nslow;
  }
  return A5X_OK;
}

int a5x_locate_device(a5x_ctx* c, const uint8_t* d_words, const uint64_t* d_woff, uint64_t nw, int mode, int mn,
                      int mx, const uint64_t* cands, uint64_t n, uint64_t* byte_off_out, void* stream) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || (nw && (!d_words || !d_woff)) || (n && (!cands || !byte_off_out))) return A5X_E_ARG;
  if (n > 0xffffffffull) return fail(c, A5X_E_ARG, "too many queries");
  int rc;
  if ((rc = check_mode(c, mode))) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  Job J;
  job_open(c, J, d_words, d_woff, nw, mode, mn, mx, stream ? (hipStream_t)stream : c->stream);
  if ((rc = job_prepare(c, J, nullptr, nullptr, false))) return rc;
  std::vector<uint64_t> q(n), res;
  for (uint64_t i = 0; i < n; i++) q[i] = std::min(cands[i], J.B.total_cands);
  if ((rc = job_locate(c, J, q, res))) return rc;
  for (uint64_t i = 0; i < n; i++) byte_off_out[i] = res[3 * i];
  return A5X_OK;
}

int a5x_split_device(a5x_ctx* c, const uint8_t* d_words, const uint64_t* d_woff, uint64_t nw, int mode, int mn,
                     int mx, const uint64_t* targets, uint32_t nt, uint64_t* cand_out, uint64_t* word_out,
                     uint64_t* ciw_out, void* stream) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || (nw && (!d_words || !d_woff)) || (nt && (!targets || !cand_out || !word_out || !ciw_out)))
    return A5X_E_ARG;
  int rc;
  if ((rc = check_mode(c, mode))) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  Job J;
  job_open(c, J, d_words, d_woff, nw, mode, mn, mx, stream ? (hipStream_t)stream : c->stream);
  if ((rc = job_prepare(c, J, nullptr, nullptr, false))) return rc;
  const uint64_t T = J.B.total_cands, TB = J.B.total_bytes;
  // lockstep binary searches: lo[i] < answer <= hi[i], byte(g) = first byte of candidate g
  std::vector<uint64_t> lo(nt), hi(nt), res;
  for (uint32_t i = 0; i < nt; i++) {
    if (targets[i] > TB) return fail(c, A5X_E_ARG, "byte target %llu past the batch's %llu bytes",
                                     (unsigned long long)targets[i], (unsigned long long)TB);
    lo[i] = ~0ull;  // "-1": byte(-1) < every target
    hi[i] = T;      // byte(T) = TB >= every target
  }
  for (int it = 0; it < 70; it++) {
    std::vector<uint64_t> q;
    std::vector<uint32_t> who;
    for (uint32_t i = 0; i < nt; i++)
      if (hi[i] - (lo[i] + 1) > 0) {  // candidates lo+1 .. hi-1 still open
        q.push_back(lo[i] + 1 + (hi[i] - lo[i] - 1) / 2);
        who.push_back(i);
      }
    if (q.empty()) break;
    if ((rc = job_locate(c, J, q, res))) return rc;
    for (size_t k = 0; k < q.size(); k++) {
      const uint32_t i = who[k];
      if (res[3 * k] >= targets[i]) hi[i] = q[k];
      else lo[i] = q[k];
    }
  }
  // the word of each split candidate and its index there: one device binary search per target
  if ((rc = grow(c, c->loc_q, nt)) || (rc = grow(c, c->loc_r, 2 * (size_t)nt))) return rc;
  HIPCHK(c, hipMemcpyAsync(c->loc_q.p, hi.data(), 8 * (size_t)nt, hipMemcpyHostToDevice, J.st));
  HIPCHK(c, a5x_launch_word_of(J.B.cand_off, nw, c->loc_q.p, nt, c->loc_r.p, c->loc_r.p + nt, J.st));
  std::vector<uint64_t> wc(2 * (size_t)nt);
  HIPCHK(c, hipMemcpyAsync(wc.data(), c->loc_r.p, 16 * (size_t)nt, hipMemcpyDeviceToHost, J.st));
  if ((rc = job_check(c, J))) return rc;
  for (uint32_t i = 0; i < nt; i++) {
    cand_out[i] = hi[i];
    word_out[i] = wc[i];
    ciw_out[i] = wc[nt + i];
  }
  return A5X_OK;
}

int a5x_digest_device(a5x_ctx* c, const uint8_t* d_out, const uint64_t* d_byte_off, uint64_t out_base, uint64_t nw,
                      uint64_t* d_digest, void* stream) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || (nw && (!d_byte_off || !d_digest))) return A5X_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  if (nw) HIPCHK(c, a5x_launch_digest(d_out, d_byte_off, out_base, nw, d_digest, st));
  HIPCHK(c, hipStreamSynchronize(st));
  return A5X_OK;
}

int a5x_keyspace(a5x_ctx* c, const uint8_t* words, const uint64_t* woff, uint64_t nw, int mode, int mn, int mx,
                 uint64_t* out_count, uint64_t* out_bytes) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || (nw && (!words || !woff))) return A5X_E_ARG;
  int rc;
  if ((rc = check_mode(c, mode))) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  const uint64_t wbytes = nw ? woff[nw] : 0;
  if ((rc = grow(c, c->s_words, wbytes + 16)) || (rc = grow(c, c->s_woff, nw + 1))) return rc;
  if (wbytes) HIPCHK(c, hipMemcpyAsync(c->s_words.p, words, wbytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->s_woff.p, woff, (nw + 1) * 8, hipMemcpyHostToDevice, c->stream));
  Batch B;
  if (mode != A5X_MODE_DEFAULT)
    rc = run_keyspace_mode(c, c->s_words.p, c->s_woff.p, nw, mode, mn, mx, nullptr, nullptr, c->stream, &B, false);
  else
    rc = run_keyspace(c, c->s_words.p, c->s_woff.p, nw, mn, mx, nullptr, nullptr, c->stream, &B, false);
  if (rc) return rc;
  if (out_count && nw) HIPCHK(c, hipMemcpyAsync(out_count, c->count.p, nw * 8, hipMemcpyDeviceToHost, c->stream));
  if (out_bytes && nw) HIPCHK(c, hipMemcpyAsync(out_bytes, c->bytes.p, nw * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return A5X_OK;
}

// The stdout path's buffers: two HBM range buffers and two pinned host buffers of cap
// bytes, the copy stream and its events (a5x_expand; a5x_stream_reserve makes them ahead).
size_t stream_cap() {
  size_t cap = (size_t)1 << 27;
  if (const char* e = getenv("A5X_HOST_CHUNK_BYTES")) cap = std::max<size_t>(4096, strtoull(e, nullptr, 10));
  return cap;
}

int stream_buffers(a5x_ctx* c, size_t cap) {
  int rc;
  if ((rc = grow(c, c->s_out[0], cap)) || (rc = grow(c, c->s_out[1], cap))) return rc;
  if (c->h_out_cap < cap) {
    for (auto& h : c->h_out)
      if (h) (void)hipHostFree(h), h = nullptr;
    c->h_out_cap = 0;
    HIPCHK(c, hipHostMalloc((void**)&c->h_out[0], cap, 0));
    HIPCHK(c, hipHostMalloc((void**)&c->h_out[1], cap, 0));
    c->h_out_cap = cap;
  }
  if (!c->cstream) HIPCHK(c, hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
  for (int i = 0; i < 2; i++) {
    if (!c->ev_exp[i]) HIPCHK(c, hipEventCreateWithFlags(&c->ev_exp[i], hipEventDisableTiming));
    if (!c->ev_cpy[i]) HIPCHK(c, hipEventCreateWithFlags(&c->ev_cpy[i], hipEventDisableTiming));
  }
  return A5X_OK;
}

int a5x_stream_reserve(a5x_ctx* c, uint64_t words, uint64_t word_bytes) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c) return A5X_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = stream_buffers(c, stream_cap()))) return rc;
  // the per-batch keyspace state of a batch of this size, and the staged words
  if ((rc = grow(c, c->s_words, word_bytes + 16)) || (rc = grow(c, c->s_woff, words + 1)) ||
      (rc = grow(c, c->count, words + 1)) || (rc = grow(c, c->bytes, words + 1)) ||
      (rc = grow(c, c->flags, words + 1)) || (rc = grow(c, c->defer, words + 1)) ||
      (rc = grow(c, c->roff, words + 1)) || (rc = grow(c, c->cplx, words + 1)) ||
      (rc = grow(c, c->slow_list, words + 1)) || (rc = grow(c, c->big_list, words + 1)) ||
      (rc = grow(c, c->glob, words + 1)) || (rc = grow(c, c->cand_off, words + 1)) ||
      (rc = grow(c, c->byte_off, words + 1)) ||
      (rc = grow(c, c->scan_tmp, a5x_scan_tmp_elems(words + 1) + 16)) ||
      (rc = grow(c, c->rec, ((words + FW_TILE - 1) / FW_TILE) * (uint64_t)FW_TILE_REC +
                                (uint64_t)ks_cplx_cap(words) * FW_RMAX + 2)))
    return rc;
  if ((rc = upload_table(c))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return A5X_OK;
}

// The stdout path (main.go:58-68): ranges of <= cap bytes expanded into two HBM buffers
// in turn; each range's D2H runs on a copy stream into a pinned buffer while the next
// range expands, and the sink consumes range k while range k + 1 is being copied.
int a5x_expand(a5x_ctx* c, const uint8_t* words, const uint64_t* woff, uint64_t nw, int mode, int mn, int mx,
               a5x_sink_fn sink, void* user, a5x_stats* stats) {
  return a5x_expand_range(c, words, woff, nw, mode, mn, mx, 0, ~0ull, sink, user, stats);
}

// a5x_expand over the batch's global candidates [cb, ce) only (the CLI's --skip / --limit
// resume cursor): the same keyspace, the ranges cut at the window's ends.
int a5x_expand_range(a5x_ctx* c, const uint8_t* words, const uint64_t* woff, uint64_t nw, int mode, int mn, int mx,
                     uint64_t cb, uint64_t ce, a5x_sink_fn sink, void* user, a5x_stats* stats) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || !sink || (nw && (!words || !woff))) return A5X_E_ARG;
  int rc;
  if ((rc = check_mode(c, mode))) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  const uint64_t wbytes = nw ? woff[nw] : 0;
  if ((rc = grow(c, c->s_words, wbytes + 16)) || (rc = grow(c, c->s_woff, nw + 1))) return rc;
  if (wbytes) HIPCHK(c, hipMemcpyAsync(c->s_words.p, words, wbytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->s_woff.p, woff, (nw + 1) * 8, hipMemcpyHostToDevice, c->stream));
  Job J;
  job_open(c, J, c->s_words.p, c->s_woff.p, nw, mode, mn, mx, c->stream);
  if ((rc = job_prepare(c, J, nullptr, nullptr, true))) return rc;
  const size_t cap = stream_cap();
  std::vector<Range> ranges;
  if ((rc = plan_ranges(c, J, cap, ranges, cb, ce))) return rc;
  if (!ranges.empty() && (rc = stream_buffers(c, cap))) return rc;
  // error word of each range, copied behind its launch (valid once its copy event fired)
  uint32_t* herr = c->h_scalars + 32;
  auto drain = [&](size_t k) -> int {  // range k has been copied: check it, hand it to the sink
    HIPCHK(c, hipEventSynchronize(c->ev_cpy[k & 1]));
    if (herr[k & 1]) return decode_dev_err(c, herr[k & 1]);
    const uint64_t nb = ranges[k].b1 - ranges[k].b0;
    if (nb && sink(user, c->h_out[k & 1], nb)) return fail(c, A5X_E_SINK, "sink returned non-zero");
    return A5X_OK;
  };
  HIPCHK(c, hipEventRecord(c->ev[1], J.st));
  for (size_t k = 0; k < ranges.size(); k++) {
    const int b = (int)(k & 1);
    if (k >= 2) HIPCHK(c, hipStreamWaitEvent(J.st, c->ev_cpy[b], 0));  // range k-2's copy left buffer b
    if ((rc = job_launch(c, J, ranges[k], c->s_out[b].p, cap))) return rc;
    HIPCHK(c, hipMemcpyAsync(herr + b, c->d_scalars + 2, 4, hipMemcpyDeviceToHost, J.st));
    HIPCHK(c, hipEventRecord(c->ev_exp[b], J.st));
    HIPCHK(c, hipStreamWaitEvent(c->cstream, c->ev_exp[b], 0));
    HIPCHK(c, hipMemcpyAsync(c->h_out[b], c->s_out[b].p, ranges[k].b1 - ranges[k].b0, hipMemcpyDeviceToHost,
                             c->cstream));
    HIPCHK(c, hipEventRecord(c->ev_cpy[b], c->cstream));
    if (k >= 1 && (rc = drain(k - 1))) return rc;
  }
  if (!ranges.empty() && (rc = drain(ranges.size() - 1))) return rc;
  HIPCHK(c, hipEventRecord(c->ev[2], J.st));
  if ((rc = job_check(c, J))) return rc;
  if (stats) {
    memset(stats, 0, sizeof *stats);
    stats->words = nw;
    stats->candidates = J.B.total_cands;  // (the whole batch; the window's: its ranges below)
    stats->bytes = J.B.total_bytes;
    if (cb != 0 || ce < J.B.total_cands) {
      stats->candidates = 0;
      stats->bytes = 0;
      for (const Range& R : ranges) stats->candidates += R.ce - R.cb, stats->bytes += R.b1 - R.b0;
    }
    float a = 0, t = 0;
    HIPCHK(c, hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
    HIPCHK(c, hipEventElapsedTime(&t, c->ev[0], c->ev[2]));
    stats->ms_keyspace = a;
    stats->ms_total = t;  // includes the D2H copies and the sink
    stats->ms_expand = t - a;
    stats->expand_launches = (uint32_t)ranges.size();
    stats->words_slow = J.B.nslow;
    stats->words_pass_b = J.B.nbig;
  }
  return A5X_OK;
}

// diagnostic builds only (-DA5X_STAMPS); A5X_E_UNSUPPORTED otherwise
int a5x_debug_stamps(unsigned long long* out16, int reset) {
  const int rc = a5x_read_stamps(out16, reset);
  return rc == 0 ? A5X_OK : (rc == -9 ? A5X_E_UNSUPPORTED : A5X_E_HIP);
}

int a5x_debug_plan_word(a5x_ctx* c, const uint8_t* word, size_t len, int mn, int mx, uint8_t* out, size_t cap,
                        uint64_t* info) {
  if (!c || !info || (!word && len) || (!out && cap)) return A5X_E_ARG;
  if (c->table.keys.empty()) return fail(c, A5X_E_NOTABLE, "no substitution table loaded");
  if (c->table_dirty || c->blob.empty()) {
    int rc = compile_table(c);
    if (rc) return rc;
  }
  info[0] = info[1] = info[2] = info[3] = 0;
  if (len > A5X_LMAX_A && mx >= 1) {
    info[2] = A5X_WF_DEFER;
    return A5X_OK;
  }
  std::vector<uint8_t> wb(word, word + len);
  wb.resize(len + 16, 0);
  GWord gw;
  gw.p = wb.data();
  const Tab T = tab_view(c->blob.data());
  const WordClass C = classify_word(gw, (u32)len, T, mn, mx, A5X_RING_A - 16);
  info[0] = C.count; info[1] = C.bytes; info[2] = C.flags;
  if (!(C.flags & A5X_WF_FAST) || C.count == 0) return A5X_OK;
  // the record exactly as k_keyspace_thread builds it, placed as a one-word window
  std::vector<u64> wrec(FX_WREC + FW_PMAX + 16, 0);
  ArraySink sk;
  sk.rec = wrec.data(); sk.np = ff_np(C.flags);
  // (diagnostics: A5X_BAL_SLACK8 overrides the balanced big-piece slack of the device
  // build, FB_BAL_SLACK8, for the window simulation in tools/window_sim.py)
  u32 slack = FB_BAL_SLACK8;
  if (const char* e = getenv("A5X_BAL_SLACK8")) slack = (u32)atoi(e);
  const Plan P = plan_word<true>(gw, (u32)len, T, sk, fb_balanced_cap(C.count + 1, slack));
  wrec[0] = fr_hdr(P.np, P.ng, P.ne, P.maxl, P.nbig, P.bstarts, P.bRp);
  wrec[FX_ZSLOT] = 0;
  if (!P.ok || P.ng != ff_ng(C.flags) || P.ne != ff_ne(C.flags) || P.np != ff_np(C.flags))
    return fail(c, A5X_E_BOUNDS, "piece plan disagrees with the keyspace fields");
  info[2] |= (uint64_t)P.nbig << 32 | (uint64_t)P.bent << 40;  // diagnostics: big pieces / entries
  if (!out) return A5X_OK;  // no out: classification and plan only
  // big pieces and their entries as the k_expand_fast window setup builds them
  u32 Rb[FB_NMAX], base[FB_NMAX], E = 0;
  std::vector<u32> be(4 * 256, 0);
  for (u32 b = 0; b < FB_NMAX; b++) {
    Rb[b] = fb_R(wrec.data(), 0, wrec[0], b);
    if (Rb[b] != frh_R(wrec[0], b)) return fail(c, A5X_E_BOUNDS, "header R of big piece %u: %u != %u", b, frh_R(wrec[0], b), Rb[b]);
    base[b] = E;
    if (b < P.nbig) E += Rb[b];
  }
  if (E != P.bent) return fail(c, A5X_E_BOUNDS, "big entries %u != plan %u", E, P.bent);
  for (u32 b = 0; b < P.nbig; b++)
    for (u32 cc = 0; cc < Rb[b]; cc++) fb_entry(wrec.data(), 0, b, cc, &be[4 * (base[b] + cc)]);
  // replay the rounds: lanes one after the other, passes 1-2 into a linear ring
  // with the head/carry hand-over and block moves exactly as the kernel does them
  if (C.bytes > cap) return fail(c, A5X_E_CAPACITY, "output buffer too small");
  const u32 RING = 2048;
  std::vector<u32> ring(RING / 4 + 4 * 64, 0xA5A5A5A5u);
  uint64_t pos = 0, B = 0;  // bytes produced / global byte of ring byte 0
  u32 carry = 0;
  const u32 nl = std::min<u32>(64, (RING - 32) / std::max<u32>(P.maxl, 1));
  auto flush = [&]() {
    const u32 nb = (u32)((pos - B) >> 4);
    if (!nb) return;
    for (uint64_t X = B; X < B + 16ull * nb; X++) out[X] = (uint8_t)(ring[(X - B) >> 2] >> (8 * ((X - B) & 3)));
    for (u32 k = 0; k < 4; k++) ring[k] = ring[4 * nb + k];
    B += 16ull * nb;
  };
  for (uint64_t rr = 0; rr < C.count; rr += nl) {
    const u32 nact = (u32)std::min<uint64_t>(nl, C.count - rr);
    u32 len[64], o[64], acc[64], pn[64], hd[64], D[64];
    u32 ent[64][FB_NMAX][4];
    u32 run = (u32)(pos - B);
    for (u32 l = 0; l < nact; l++) {
      u32 n = (u32)(rr + l + 1);
      len[l] = 0;
      for (u32 b = 0; b < FB_NMAX; b++) {
        const u32 q = Rb[b] > 1 ? (u32)(((u64)n * fr_magic(Rb[b])) >> 32) : n;
        const u32 d = n - q * Rb[b];
        n = q;
        for (u32 k = 0; k < 4; k++) ent[l][b][k] = b < P.nbig ? be[4 * (base[b] + d) + k] : 0u;
        len[l] += ent[l][b][3] >> 24;
      }
      o[l] = run;
      run += len[l];
    }
    for (u32 l = 0; l < nact; l++) {
      pn[l] = o[l] & 3u; D[l] = o[l] >> 2; acc[l] = 0; hd[l] = 0;
      u32 pv = l == 0 ? (carry << ((32u - 8u * pn[l]) & 31u)) : 0u;
      bool hp = l != 0 && pn[l] != 0;
      for (u32 b = 0; b < FB_NMAX; b++) fb_put(ent[l][b], pv, pn[l], D[l], hp, hd[l], acc[l], ring.data(), RING / 4 + 4 * l);
    }
    for (u32 l = 0; l < nact; l++)
      ring[(l + 1 < nact && pn[l]) ? D[l] : RING / 4 + 4 * l] = acc[l] | (l + 1 < nact ? hd[l + 1] : 0u);
    carry = acc[nact - 1];
    pos = B + run;
    flush();
  }
  if (pos & 3) ring[(u32)(pos - B) >> 2] = carry;
  flush();
  for (uint64_t X = B; X < pos; X++) out[X] = (uint8_t)(ring[(X - B) >> 2] >> (8 * ((X - B) & 3)));
  if (pos != C.bytes) return fail(c, A5X_E_BOUNDS, "replayed %llu bytes, keyspace says %llu",
                                  (unsigned long long)pos, (unsigned long long)C.bytes);
  info[3] = pos;
  return A5X_OK;
}

int a5x_set_targets(a5x_ctx* c, int algo, const uint8_t* dig, uint64_t n) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || (n && !dig)) return A5X_E_ARG;
  if (algo != A5X_ALGO_MD5 && algo != A5X_ALGO_NTLM) return fail(c, A5X_E_ARG, "bad digest algorithm %d", algo);
  HIPCHK(c, hipSetDevice(c->device));
  // prefilter: >= 64 bits per target (false-positive rate <= 1/64), table: load <= 1/2
  uint32_t bm_log2 = 16;
  while (bm_log2 < 32 && (1ull << bm_log2) < n * 64) bm_log2++;
  // (test hook: force the prefilter size, e.g. the 2^32-bit filter of > 2^26 targets)
  if (const char* e = getenv("A5X_TARGET_BM_LOG2")) bm_log2 = std::max(16u, std::min(32u, (uint32_t)atoi(e)));
  uint64_t tsz = 16;
  while (tsz < 2 * n) tsz <<= 1;
  std::vector<uint32_t> bm((1ull << bm_log2) / 32, 0);
  std::vector<uint4> tab(tsz);
  memset(tab.data(), 0, tsz * sizeof(uint4));
  uint32_t has_zero = 0;
  const uint64_t tmask = tsz - 1;
  for (uint64_t i = 0; i < n; i++) {
    uint32_t d[4];
    memcpy(d, dig + 16 * i, 16);
    if ((d[0] | d[1] | d[2] | d[3]) == 0) { has_zero = 1; continue; }
    const uint32_t bi = d[0] & (uint32_t)((1ull << bm_log2) - 1);
    if (MD_BLOOM2) {  // (a5x_md.h md_prefilter: the 64-bit word of bi, two bits from word 3)
      const uint64_t m = md_bloom_bits(d[3]);
      bm[(bi >> 6) * 2] |= (uint32_t)m;
      bm[(bi >> 6) * 2 + 1] |= (uint32_t)(m >> 32);
    } else {
      bm[bi >> 5] |= 1u << (bi & 31);
    }
    for (uint64_t slot = tgt_slot(d, tmask);; slot = (slot + 1) & tmask) {
      uint4& e = tab[slot];
      if (e.x == d[0] && e.y == d[1] && e.z == d[2] && e.w == d[3]) break;  // duplicate
      if ((e.x | e.y | e.z | e.w) == 0) { e = make_uint4(d[0], d[1], d[2], d[3]); break; }
    }
  }
  int rc;
  if ((rc = grow(c, c->t_bitmap, bm.size())) || (rc = grow(c, c->t_table, tsz))) return rc;
  HIPCHK(c, hipMemcpy(c->t_bitmap.p, bm.data(), bm.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->t_table.p, tab.data(), tsz * sizeof(uint4), hipMemcpyHostToDevice));
  c->t_algo = algo;
  c->n_targets = n;
  c->t_bm_log2 = bm_log2;
  c->t_tmask = tmask;
  c->t_has_zero = has_zero;
  return A5X_OK;
}

int a5x_expand_digest_device(a5x_ctx* c, const uint8_t* d_words, const uint64_t* d_woff, uint64_t nw, int mode,
                             int mn, int mx, uint64_t scratch_bytes, a5x_hit* hits, uint64_t hit_cap,
                             uint64_t* n_hits, a5x_stats* stats, void* stream) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || (nw && (!d_words || !d_woff)) || (hit_cap && !hits)) return A5X_E_ARG;
  if (c->t_algo < 0) return fail(c, A5X_E_ARG, "no target set (a5x_set_targets)");
  int rc;
  if ((rc = check_mode(c, mode))) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  const bool fused = !getenv("A5X_NO_FUSED_DIGEST");
  return expand_digest(c, d_words, d_woff, nw, mode, mn, mx, 0, ~0ull, scratch_bytes, hits, hit_cap, n_hits, stats,
                       stream ? (hipStream_t)stream : c->stream, fused);
}

int a5x_expand_digest_range_device(a5x_ctx* c, const uint8_t* d_words, const uint64_t* d_woff, uint64_t nw, int mode,
                                   int mn, int mx, uint64_t cand_begin, uint64_t cand_end, uint64_t scratch_bytes,
                                   a5x_hit* hits, uint64_t hit_cap, uint64_t* n_hits, a5x_stats* stats, void* stream) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || (nw && (!d_words || !d_woff)) || (hit_cap && !hits) || cand_end < cand_begin) return A5X_E_ARG;
  if (c->t_algo < 0) return fail(c, A5X_E_ARG, "no target set (a5x_set_targets)");
  int rc;
  if ((rc = check_mode(c, mode))) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  const bool fused = !getenv("A5X_NO_FUSED_DIGEST");
  return expand_digest(c, d_words, d_woff, nw, mode, mn, mx, cand_begin, cand_end, scratch_bytes, hits, hit_cap,
                       n_hits, stats, stream ? (hipStream_t)stream : c->stream, fused);
}

int a5x_expand_digest(a5x_ctx* c, const uint8_t* words, const uint64_t* woff, uint64_t nw, int mode, int mn, int mx,
                      a5x_hit* hits, uint64_t hit_cap, uint64_t* n_hits, a5x_stats* stats) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || (nw && (!words || !woff))) return A5X_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const uint64_t wbytes = nw ? woff[nw] : 0;
  int rc;
  if ((rc = grow(c, c->s_words, wbytes + 16)) || (rc = grow(c, c->s_woff, nw + 1))) return rc;
  if (wbytes) HIPCHK(c, hipMemcpyAsync(c->s_words.p, words, wbytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->s_woff.p, woff, (nw + 1) * 8, hipMemcpyHostToDevice, c->stream));
  return a5x_expand_digest_device(c, c->s_words.p, c->s_woff.p, nw, mode, mn, mx, 0, hits, hit_cap, n_hits, stats,
                                  c->stream);
}

int a5x_digest_lines_device(a5x_ctx* c, int algo, const uint8_t* d_lines, uint64_t nbytes, uint8_t* d_dig,
                            uint64_t cap, uint64_t* n_lines, void* stream) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || (nbytes && !d_lines)) return A5X_E_ARG;
  if (algo != A5X_ALGO_MD5 && algo != A5X_ALGO_NTLM) return fail(c, A5X_E_ARG, "bad digest algorithm %d", algo);
  if (((uintptr_t)d_lines & 15u) != 0) return fail(c, A5X_E_ARG, "d_lines must be 16-byte aligned");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  if (n_lines) *n_lines = 0;
  if (!nbytes) return A5X_OK;
  HIPCHK(c, hipMemsetAsync(c->d_scalars, 0, 64, st));
  A5xDigLaunch D = dig_launch(c);
  D.algo = algo;
  D.out = d_lines;
  D.nbytes = nbytes;
  uint64_t lines = 0;
  int rc;
  if ((rc = dig_block_prefix(c, D, st, &lines))) return rc;
  if (n_lines) *n_lines = lines;
  if (lines > cap || !d_dig)
    return fail(c, A5X_E_CAPACITY, "%llu lines, digest buffer has room for %llu", (unsigned long long)lines,
                (unsigned long long)cap);
  D.dig_out = d_dig;
  HIPCHK(c, a5x_launch_digest_stream(D, 2, dig_grid(c), st));
  HIPCHK(c, hipMemcpyAsync(c->h_scalars, c->d_scalars, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  return decode_dev_err(c, c->h_scalars[2]);
}

int a5x_partition(const uint64_t* prefix, uint64_t n, uint32_t parts, uint64_t* split) {
  if (!prefix || !split || parts == 0) return A5X_E_ARG;
  const uint64_t total = prefix[n];
  split[0] = 0;
  for (uint32_t r = 1; r < parts; r++) {
    const unsigned __int128 target = (unsigned __int128)total * r / parts;
    // first word i whose start offset >= target
    uint64_t lo = split[r - 1], hi = n;
    while (lo < hi) {
      const uint64_t mid = lo + (hi - lo) / 2;
      if ((unsigned __int128)prefix[mid] < target) lo = mid + 1; else hi = mid;
    }
    split[r] = lo;
  }
  split[parts] = n;
  return A5X_OK;
}

// ---- hashcat-style hit output (README.MD:74-106, :168) ------------
// hashcat's outfile auto-hex convention, restated (hashcat is not part of the
// reference): a plain is written as $HEX[lowercase hex] when it is not valid UTF-8
// (Go utf8.Valid rules), contains a control byte (< 0x20 or 0x7f, which would break
// the "hash:plain" line), or itself has the $HEX[...] form.
static bool plain_needs_hex(const uint8_t* p, size_t n) {
  if (n >= 6 && memcmp(p, "$HEX[", 5) == 0 && p[n - 1] == ']') return true;
  for (size_t i = 0; i < n;) {
    if (p[i] < 0x20 || p[i] == 0x7f) return true;
    int sz;
    const int r = a5x::gosem::decode_rune(p + i, n - i, &sz);
    if (r == a5x::gosem::kRuneError && sz == 1) return true;  // invalid byte (a literal U+FFFD has sz 3)
    i += (size_t)sz;
  }
  return false;
}

static void append_plain(std::string& o, const uint8_t* p, size_t n) {
  static const char* hx = "0123456789abcdef";
  if (!plain_needs_hex(p, n)) {
    o.append((const char*)p, n);
    return;
  }
  o += "$HEX[";
  for (size_t i = 0; i < n; i++) {
    o += hx[p[i] >> 4];
    o += hx[p[i] & 15];
  }
  o += ']';
}

int a5x_format_plain(const uint8_t* plain, size_t len, uint8_t* out, size_t cap, size_t* out_len) {
  if ((!plain && len) || !out_len) return A5X_E_ARG;
  std::string o;
  append_plain(o, plain, len);
  *out_len = o.size();
  if (!out || cap < o.size()) return out ? A5X_E_CAPACITY : A5X_OK;
  memcpy(out, o.data(), o.size());
  return A5X_OK;
}

int a5x_format_hits(a5x_ctx* c, const uint8_t* words, const uint64_t* woff, uint64_t nw, int mode, int mn, int mx,
                    const a5x_hit* hits, uint64_t n_hits, a5x_sink_fn sink, void* user) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || !sink || (n_hits && (!hits || !words || !woff))) return A5X_E_ARG;
  if (!n_hits) return A5X_OK;
  int rc;
  if ((rc = check_mode(c, mode))) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  // The hit words, once each, as a sub-batch; only the hit candidates themselves are
  // regenerated on the device (located, then expanded as single-candidate ranges, or
  // one range per run of nearby hits), never a hit word's whole keyspace: a word's
  // output may exceed host memory and 2^32 bytes.
  std::vector<uint64_t> uw(n_hits);
  for (uint64_t h = 0; h < n_hits; h++) {
    if (hits[h].word >= nw) return fail(c, A5X_E_ARG, "hit word index beyond the batch");
    uw[h] = hits[h].word;
  }
  std::sort(uw.begin(), uw.end());
  uw.erase(std::unique(uw.begin(), uw.end()), uw.end());
  std::vector<uint8_t> sb;
  std::vector<uint64_t> so(1, 0);
  for (uint64_t w : uw) {
    sb.insert(sb.end(), words + woff[w], words + woff[w + 1]);
    so.push_back(sb.size());
  }
  sb.resize(sb.size() + 16, 0);
  const uint64_t m = uw.size();
  if ((rc = grow(c, c->s_words, sb.size())) || (rc = grow(c, c->s_woff, m + 1))) return rc;
  HIPCHK(c, hipMemcpyAsync(c->s_words.p, sb.data(), sb.size(), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->s_woff.p, so.data(), (m + 1) * 8, hipMemcpyHostToDevice, c->stream));
  Job J;
  job_open(c, J, c->s_words.p, c->s_woff.p, m, mode, mn, mx, c->stream);
  if ((rc = job_prepare(c, J, nullptr, nullptr, false))) return rc;
  std::vector<uint64_t> coff(m + 1);
  HIPCHK(c, hipMemcpyAsync(coff.data(), J.B.cand_off, (m + 1) * 8, hipMemcpyDeviceToHost, J.st));
  HIPCHK(c, hipStreamSynchronize(J.st));
  // global candidate index (in the sub-batch) of every hit
  std::vector<uint64_t> g(n_hits);
  for (uint64_t h = 0; h < n_hits; h++) {
    const size_t k = (size_t)(std::lower_bound(uw.begin(), uw.end(), hits[h].word) - uw.begin());
    if (hits[h].cand >= coff[k + 1] - coff[k])
      return fail(c, A5X_E_ARG, "hit candidate index beyond its word's keyspace");
    g[h] = coff[k] + hits[h].cand;
  }
  std::vector<uint64_t> ug(g);
  std::sort(ug.begin(), ug.end());
  ug.erase(std::unique(ug.begin(), ug.end()), ug.end());
  // runs of hit candidates: a run spans at most 4096 candidates (its bytes are checked
  // after the locate: a run over 1 MiB is split into single-candidate ranges)
  struct Run { size_t a, b; };  // ug[a..b)
  std::vector<Run> runs;
  for (size_t i = 0; i < ug.size();) {
    size_t j = i + 1;
    while (j < ug.size() && ug[j] - ug[i] < 4096) j++;
    runs.push_back({i, j});
    i = j;
  }
  std::vector<uint64_t> q;
  for (auto& r : runs) { q.push_back(ug[r.a]); q.push_back(ug[r.b - 1] + 1); }
  std::vector<uint64_t> loc;
  if ((rc = job_locate(c, J, q, loc))) return rc;
  std::vector<Range> ranges;  // one per run, or per candidate of an oversize run
  std::vector<std::pair<size_t, size_t>> rcand;  // ug[first, last) covered by each range
  std::vector<uint64_t> q2;
  std::vector<size_t> split_runs;
  for (size_t r = 0; r < runs.size(); r++) {
    const uint64_t* lb = &loc[3 * (2 * r)];
    const uint64_t* le = &loc[3 * (2 * r + 1)];
    if (le[0] - lb[0] <= (1u << 20) || runs[r].b - runs[r].a == 1) {
      ranges.push_back(range_of(J, ug[runs[r].a], ug[runs[r].b - 1] + 1, lb, le));
      rcand.push_back({runs[r].a, runs[r].b});
    } else {
      split_runs.push_back(r);
      for (size_t i = runs[r].a; i < runs[r].b; i++) { q2.push_back(ug[i]); q2.push_back(ug[i] + 1); }
    }
  }
  if (!q2.empty()) {
    std::vector<uint64_t> loc2;
    if ((rc = job_locate(c, J, q2, loc2))) return rc;
    size_t t = 0;
    for (size_t r : split_runs)
      for (size_t i = runs[r].a; i < runs[r].b; i++, t++) {
        ranges.push_back(range_of(J, ug[i], ug[i] + 1, &loc2[3 * (2 * t)], &loc2[3 * (2 * t + 1)]));
        rcand.push_back({i, i + 1});
      }
  }
  // expand every range into the staging buffer and cut out the hit candidates
  std::vector<std::string> plain(ug.size());
  std::vector<uint8_t> hb;
  for (size_t r = 0; r < ranges.size(); r++) {
    const Range& R = ranges[r];
    const uint64_t nb = R.b1 - R.b0;
    if ((rc = grow(c, c->s_out[0], nb + 64))) return rc;
    if ((rc = job_launch(c, J, R, c->s_out[0].p, nb + 64))) return rc;
    hb.resize(nb);
    HIPCHK(c, hipMemcpyAsync(hb.data(), c->s_out[0].p, nb, hipMemcpyDeviceToHost, J.st));
    if ((rc = job_check(c, J))) return rc;
    // the range's lines are candidates R.cb, R.cb + 1, ... in order
    size_t want = rcand[r].first;
    uint64_t cand = R.cb, p0 = 0;
    for (uint64_t x = 0; x < nb && want < rcand[r].second; x++) {
      if (hb[x] != '\n') continue;
      if (cand == ug[want]) plain[want++].assign((const char*)hb.data() + p0, (size_t)(x - p0));
      cand++;
      p0 = x + 1;
    }
    if (want != rcand[r].second) return fail(c, A5X_E_HIP, "hit candidates not found in their located range");
  }
  static const char* hx = "0123456789abcdef";
  std::string o;
  for (uint64_t h = 0; h < n_hits; h++) {
    const size_t k = (size_t)(std::lower_bound(ug.begin(), ug.end(), g[h]) - ug.begin());
    for (int i = 0; i < 16; i++) {
      o += hx[hits[h].digest[i] >> 4];
      o += hx[hits[h].digest[i] & 15];
    }
    o += ':';
    append_plain(o, (const uint8_t*)plain[k].data(), plain[k].size());
    o += '\n';
    if (o.size() >= (1u << 20) || h + 1 == n_hits) {
      if (sink(user, (const uint8_t*)o.data(), o.size())) return fail(c, A5X_E_SINK, "sink returned non-zero");
      o.clear();
    }
  }
  return A5X_OK;
}

int a5x_dev_alloc(a5x_ctx* c, void** p, size_t bytes) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c || !p) return A5X_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  hipError_t e = hipMalloc(p, bytes ? bytes : 16);
  if (e != hipSuccess) return fail(c, A5X_E_NOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
  return A5X_OK;
}
int a5x_dev_free(a5x_ctx* c, void* p) {
  if (!c) return A5X_E_ARG;
  if (p) HIPCHK(c, hipFree(p));
  return A5X_OK;
}
int a5x_memcpy_h2d(a5x_ctx* c, void* dst, const void* src, size_t bytes) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c) return A5X_E_ARG;
  HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return A5X_OK;
}
int a5x_memcpy_d2h(a5x_ctx* c, void* dst, const void* src, size_t bytes) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c) return A5X_E_ARG;
  HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return A5X_OK;
}
int a5x_synchronize(a5x_ctx* c) {
  if (c && c->device < 0) return fail(c, A5X_E_HIP, "host-only context (device -1) cannot run kernels");
  if (!c) return A5X_E_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return A5X_OK;
}

}  // extern "C"
