// a5x_cli.cpp -- `a5x_generator`: C++ replica of the reference CLI (main.go:17-100)
// on top of liba5x.  Same flags (main.go:18-26, kong conventions), same
// "cand\n" stdout format (main.go:66).  Used by tests and benchmarks because the
// Go toolchain is absent here; the Go CLI itself binds liba5x through the cgo
// stub shown in INTEGRATION.md.
//
//   a5x_generator <dict-file> -t <table> [-t <table> ...] [-m N] [-x N]
//                 [--threads N] [-s] [-r] [--device N]
//                 [--hashes <file> [--algo md5|ntlm]]
//                 [--skip N] [--limit N] [--keyspace]
//
// --hashes (a5x extension): instead of printing the candidates for a
// hashcat pipe (README.MD:69), hash them on the GPU (fused MD5 / NTLM + lookup) against
// the hex digests of <file> and print what hashcat would report, "hash:plain" (plains
// that hashcat would hexify as $HEX[...]), each target once, at its first candidate in
// stream order (README.MD:74-106, :168).
//
// --skip / --limit / --keyspace (a5x extension, SURVEY §5 checkpoint / resume): the
// stream's candidate order does not depend on batching (a word's candidates are
// numbered alike in any batch), so a candidate index is a resume cursor: --skip N
// --limit M prints candidates [N, N + M) of the full stream, as hashcat's -s / -l would
// on the pipe; --keyspace prints the number of candidates the run would print.  Whole
// batches before the window cost only their keyspace pass.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "a5x.h"
#include "a5x_gosem.h"

static void usage(FILE* f) {
  fprintf(f,
          "Usage: a5_generator --table-files=TABLE-FILES,... <dict-file> [flags]\n\n"
          "Generates word variations based on a substitution table. v0.2\n\n"
          "Arguments:\n  <dict-file>    Path to dictionary file\n\n"
          "Flags:\n"
          "  -h, --help                        Show context-sensitive help.\n"
          "  -t, --table-files=TABLE-FILES,... Path to substitution table (multiple possible, sequential)\n"
          "  -m, --table-min=0                 Minimum substitutions\n"
          "  -x, --table-max=15                Maximum substitutions\n"
          "      --threads=-1                  Number of threads (accepted; the GPU needs none)\n"
          "  -s, --substitute-all              Substitution Cipher, see Transliteration Attack\n"
          "  -r, --reverse-sub                 Reverse substitution direction\n"
          "      --device=0                    GPU ordinal (a5x extension)\n"
          "      --hashes=FILE                 Crack: print hash:plain for the digests in FILE (a5x extension)\n"
          "      --algo=md5                    Digest of --hashes: md5 (hashcat -m 0) or ntlm (-m 1000)\n"
          "      --skip=0                      Resume: start at candidate N of the stream (a5x extension)\n"
          "      --limit=N                     Print at most N candidates (a5x extension)\n"
          "      --keyspace                    Print the number of candidates and exit (a5x extension)\n");
}

// ---------------------------------------------------------------------------
// Dictionary stream (main.go:52-56, 72-74): bufio.Scanner + ScanLines over the file in
// bounded chunks -- LF split, one trailing CR dropped, a final unterminated line kept,
// and the first line with no '\n' in 64 KiB (bufio.ErrTooLong) silently ends the input,
// as the reference never checks scanner.Err().  At most one chunk of file bytes plus one
// batch per pipeline slot is resident, whatever the dictionary size.
// ---------------------------------------------------------------------------
struct DictStream {
  FILE* f = nullptr;
  std::vector<uint8_t> buf;
  size_t pos = 0, end = 0;
  bool eof = false, stop = false;
  explicit DictStream(FILE* fp, size_t chunk = (size_t)64 << 20) : f(fp), buf(chunk + a5x::gosem::kMaxScanToken) {}
  // keep >= 64 KiB (or the rest of the file) past pos, so a line is cut exactly where
  // the whole-file scanner would cut it
  void fill() {
    if (eof || end - pos >= a5x::gosem::kMaxScanToken) return;
    memmove(buf.data(), buf.data() + pos, end - pos);
    end -= pos;
    pos = 0;
    while (!eof && end < buf.size()) {
      const size_t r = fread(buf.data() + end, 1, buf.size() - end, f);
      if (r == 0) eof = true;
      end += r;
    }
  }
  // the next batch: up to max_words words / about max_bytes bytes (+16 B pad)
  bool next(std::vector<uint8_t>& words, std::vector<uint64_t>& off, uint64_t max_words, size_t max_bytes) {
    words.clear();
    off.assign(1, 0);
    while (!stop && off.size() - 1 < max_words && words.size() < max_bytes) {
      fill();
      const uint8_t* line;
      size_t len;
      const int r = a5x::gosem::scan_line(buf.data(), end, &pos, &line, &len);
      if (r <= 0) { stop = true; break; }  // EOF, or ErrTooLong (silently the end, main.go:73)
      words.insert(words.end(), line, line + len);
      off.push_back(words.size());
    }
    words.resize(words.size() + 16, 0);
    return off.size() > 1;
  }
};

// ---------------------------------------------------------------------------
// Batch pipeline: two liba5x contexts on the device, each driven by its own thread,
// take alternate batches; batch k + 1's upload, keyspace and first range run while
// batch k's output is still streaming to stdout.  Output stays in batch order: a
// batch's sink waits for its turn (the reference's order across words is arbitrary,
// main.go:77, but a deterministic stream is easier to check).
// ---------------------------------------------------------------------------
struct Turn {
  std::mutex mu;
  std::condition_variable cv;
  uint64_t turn = 0;
  void wait(uint64_t k) {
    std::unique_lock<std::mutex> l(mu);
    cv.wait(l, [&] { return turn == k; });
  }
  void done(uint64_t k) {
    std::lock_guard<std::mutex> l(mu);
    turn = k + 1;
    cv.notify_all();
  }
};

// host timeline (A5X_CLI_TIMELINE=1): milliseconds since main() per event, to stderr
static const auto g_t0 = std::chrono::steady_clock::now();
static bool g_tl = false;
static double ms_now() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - g_t0).count();
}
#define TL(...)                                \
  do {                                         \
    if (g_tl) {                                \
      fprintf(stderr, "[tl %9.2f] ", ms_now()); \
      fprintf(stderr, __VA_ARGS__);            \
      fputc('\n', stderr);                     \
    }                                          \
  } while (0)

struct SinkCtx {
  Turn* t;
  uint64_t k;
  bool waited;
  const std::atomic<int>* failed;  // a failed earlier batch: write nothing more
  uint64_t bytes;
};

static int sink_ordered(void* user, const uint8_t* data, size_t len) {
  SinkCtx* s = (SinkCtx*)user;
  if (!s->waited) {
    TL("batch %llu: first range ready, waiting for its turn", (unsigned long long)s->k);
    s->t->wait(s->k);
    TL("batch %llu: streaming", (unsigned long long)s->k);
    s->waited = true;
  }
  if (s->failed->load()) return 1;
  s->bytes += len;
  return fwrite(data, 1, len, stdout) == len ? 0 : 1;
}

static int sink_stdout(void* user, const uint8_t* data, size_t len) {
  (void)user;
  return fwrite(data, 1, len, stdout) == len ? 0 : 1;
}

static int hexv(int c) {
  return c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
}

// target digests: one hex digest per line (32 hex digits; anything after them, e.g. a
// ":plain" of a potfile line, is ignored); other lines are counted and skipped.  Whole
// lines of any length (getline): a long potfile plain is one line, never a continuation
// piece read as a target.
static int load_targets(a5x_ctx* ctx, const char* path, int algo) {
  FILE* f = fopen(path, "rb");
  if (!f) return A5X_E_IO;
  std::vector<uint8_t> dig;
  char* line = nullptr;
  size_t cap = 0;
  ssize_t n;
  uint64_t bad = 0;
  while ((n = getline(&line, &cap, f)) >= 0) {
    size_t k = 0;
    uint8_t d[16];
    for (; k < 32 && k < (size_t)n; k++) {
      const int v = hexv((unsigned char)line[k]);
      if (v < 0) break;
      if (k & 1) d[k / 2] |= (uint8_t)v; else d[k / 2] = (uint8_t)(v << 4);
    }
    const char t = (size_t)n > 32 ? line[32] : 0;
    if (k == 32 && (t == 0 || t == '\n' || t == '\r' || t == ':')) dig.insert(dig.end(), d, d + 16);
    else if (n > 0 && line[0] != '\n' && line[0] != '\r') bad++;
  }
  free(line);
  fclose(f);
  if (bad) fprintf(stderr, "a5_generator: %llu line(s) of %s are not 32-hex-digit hashes (skipped)\n",
                   (unsigned long long)bad, path);
  return a5x_set_targets(ctx, algo, dig.empty() ? nullptr : dig.data(), dig.size() / 16);
}

static bool parse_u64(const char* s, uint64_t* out) {
  char* e;
  errno = 0;
  // digits only: strtoull would skip leading blanks and negate a '-' (" -3" -> 2^64 - 3)
  if (*s < '0' || *s > '9') return false;
  const unsigned long long v = strtoull(s, &e, 10);
  if (*e || errno) return false;
  *out = v;
  return true;
}

static bool parse_int(const char* s, int* out) {
  char* e;
  long v = strtol(s, &e, 10);
  if (!*s || *e) return false;
  *out = (int)v;
  return true;
}

// --skip / --limit / --keyspace: one context, batches in order; each batch's keyspace
// gives its candidate total T, so the window [skip, skip + limit) maps to a candidate
// range of the batches it meets (a5x_expand_range), and the batches past it are not read.
static int run_cursor(const std::string& dict, const std::vector<std::string>& tables, int device, int mode, int tmin,
                      int tmax, uint64_t B, size_t BB, size_t chunk, uint64_t skip, uint64_t limit, bool keyspace_only) {
  a5x_ctx* ctx = nullptr;
  int rc = a5x_create(device, &ctx);
  if (rc) { fprintf(stderr, "a5_generator: no usable GPU (a5x_create=%d)\n", rc); return 1; }
  for (auto& t : tables)
    if ((rc = a5x_load_table_file(ctx, t.c_str()))) {
      fprintf(stderr, "%s\n", a5x_last_error(ctx));  // log.Fatal (main.go:43-45)
      a5x_destroy(ctx);
      return 1;
    }
  FILE* f = fopen(dict.c_str(), "rb");
  if (!f) { perror(dict.c_str()); a5x_destroy(ctx); return 1; }
  const uint64_t end = limit > ~0ull - skip ? ~0ull : skip + limit;  // (saturating)
  DictStream ds(f, chunk);
  std::vector<uint8_t> words;
  std::vector<uint64_t> off, cnt;
  uint64_t G = 0;  // stream candidates before this batch
  bool ovf = false;
  while (rc == 0 && (keyspace_only || G < end) && ds.next(words, off, B, BB)) {
    const uint64_t nb = off.size() - 1;
    cnt.assign(nb, 0);
    if ((rc = a5x_keyspace(ctx, words.data(), off.data(), nb, mode, tmin, tmax, cnt.data(), nullptr))) break;
    uint64_t T = 0;
    for (uint64_t x : cnt) {
      ovf |= T + x < T;
      T += x;
    }
    if (!keyspace_only) {
      const uint64_t lo = skip > G ? std::min(T, skip - G) : 0, hi = end - G < T ? end - G : T;
      if (lo < hi)
        rc = a5x_expand_range(ctx, words.data(), off.data(), nb, mode, tmin, tmax, lo, hi, sink_stdout, nullptr,
                              nullptr);
    }
    ovf |= G + T < G;
    G += T;
  }
  fclose(f);
  if (rc == 0 && keyspace_only) {
    if (ovf) { fprintf(stderr, "a5_generator: the keyspace exceeds 2^64 - 1 candidates\n"); rc = A5X_E_OVERFLOW; }
    else printf("%llu\n", (unsigned long long)G);
  }
  if (fflush(stdout) != 0 || ferror(stdout)) {
    if (!rc) fprintf(stderr, "a5_generator: writing stdout: %s\n", strerror(errno));
    rc = rc ? rc : 1;
  } else if (rc && rc != A5X_E_OVERFLOW) {
    fprintf(stderr, "a5_generator: %s\n", a5x_last_error(ctx));
  }
  a5x_destroy(ctx);
  return rc ? 2 : 0;
}

int main(int argc, char** argv) {
  std::vector<std::string> tables;
  std::string dict;
  int tmin = 0, tmax = 15, threads = -1, device = 0, algo = A5X_ALGO_MD5;
  std::string hashes;
  bool suball = false, rev = false, keyspace_only = false, cursor = false;
  uint64_t skip = 0, limit = ~0ull;
  auto need = [&](int& i, const char* flag) -> const char* {
    if (i + 1 >= argc) {
      fprintf(stderr, "a5_generator: error: %s: expected value\n", flag);
      usage(stderr);
      exit(80);
    }
    return argv[++i];
  };
  auto add_tables = [&](const char* v) {  // kong []string flags split on ','
    std::string s(v);
    size_t p = 0;
    while (true) {
      size_t q = s.find(',', p);
      tables.push_back(s.substr(p, q == std::string::npos ? std::string::npos : q - p));
      if (q == std::string::npos) break;
      p = q + 1;
    }
  };
  for (int i = 1; i < argc; i++) {
    const char* a = argv[i];
    std::string s(a);
    auto val_of = [&](const char* flag) -> const char* {
      size_t eq = s.find('=');
      if (eq != std::string::npos) return a + eq + 1;
      return need(i, flag);
    };
    int v;
    if (s == "-h" || s == "--help") { usage(stdout); return 0; }
    else if (s == "-t" || s.rfind("--table-files", 0) == 0) add_tables(val_of("--table-files"));
    else if (s == "-m" || s.rfind("--table-min", 0) == 0) {
      if (!parse_int(val_of("--table-min"), &v)) { fprintf(stderr, "a5_generator: error: --table-min: bad int\n"); return 80; }
      tmin = v;
    } else if (s == "-x" || s.rfind("--table-max", 0) == 0) {
      if (!parse_int(val_of("--table-max"), &v)) { fprintf(stderr, "a5_generator: error: --table-max: bad int\n"); return 80; }
      tmax = v;
    } else if (s.rfind("--threads", 0) == 0) {
      if (!parse_int(val_of("--threads"), &v)) { fprintf(stderr, "a5_generator: error: --threads: bad int\n"); return 80; }
      threads = v;
    } else if (s.rfind("--device", 0) == 0) {
      if (!parse_int(val_of("--device"), &v)) { fprintf(stderr, "a5_generator: error: --device: bad int\n"); return 80; }
      device = v;
    } else if (s.rfind("--hashes", 0) == 0) {
      hashes = val_of("--hashes");
    } else if (s.rfind("--algo", 0) == 0) {
      std::string v = val_of("--algo");
      if (v == "md5" || v == "0") algo = A5X_ALGO_MD5;
      else if (v == "ntlm" || v == "1000") algo = A5X_ALGO_NTLM;
      else { fprintf(stderr, "a5_generator: error: --algo: md5 or ntlm\n"); return 80; }
    } else if (s.rfind("--skip", 0) == 0) {
      if (!parse_u64(val_of("--skip"), &skip)) { fprintf(stderr, "a5_generator: error: --skip: bad count\n"); return 80; }
      cursor = true;
    } else if (s.rfind("--limit", 0) == 0) {
      if (!parse_u64(val_of("--limit"), &limit)) { fprintf(stderr, "a5_generator: error: --limit: bad count\n"); return 80; }
      cursor = true;
    } else if (s == "--keyspace") keyspace_only = true;
    else if (s == "--substitute-all") suball = true;
    else if (s == "--reverse-sub") rev = true;
    else if (s.size() > 1 && s[0] == '-' && s[1] != '-') {
      bool ok = true;  // combined boolean shorts, e.g. -sr
      for (size_t k = 1; k < s.size(); k++) {
        if (s[k] == 's') suball = true;
        else if (s[k] == 'r') rev = true;
        else ok = false;
      }
      if (!ok) { fprintf(stderr, "a5_generator: error: unknown flag %s\n", a); usage(stderr); return 80; }
    } else if (dict.empty()) dict = s;
    else { fprintf(stderr, "a5_generator: error: unexpected argument %s\n", a); usage(stderr); return 80; }
  }
  (void)threads;
  if (tables.empty()) { fprintf(stderr, "a5_generator: error: missing flags: --table-files=TABLE-FILES,...\n"); usage(stderr); return 80; }
  if (dict.empty()) { fprintf(stderr, "a5_generator: error: expected \"<dict-file>\"\n"); usage(stderr); return 80; }

  g_tl = getenv("A5X_CLI_TIMELINE") != nullptr;
  TL("main");
  const int mode = (suball ? A5X_MODE_SUBALL : A5X_MODE_DEFAULT) + (rev ? 1 : 0);
  uint64_t B = 1u << 22;           // words per batch
  size_t BB = (size_t)64 << 20;    // word bytes per batch
  size_t chunk = (size_t)64 << 20; // dictionary bytes read at a time
  // (test hooks: small batches / chunks exercise the pipeline and the chunk edges)
  if (const char* e = getenv("A5X_CLI_BATCH")) B = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
  if (const char* e = getenv("A5X_CLI_CHUNK")) chunk = std::max<size_t>(1, strtoull(e, nullptr, 10));
  static char obuf[1 << 22];
  setvbuf(stdout, obuf, _IOFBF, sizeof obuf);
  if (!hashes.empty() && (cursor || keyspace_only)) {
    fprintf(stderr, "a5_generator: error: --skip / --limit / --keyspace select the candidate stream, not --hashes\n");
    return 80;
  }
  if (hashes.empty() && (cursor || keyspace_only)) return run_cursor(dict, tables, device, mode, tmin, tmax, B, BB, chunk,
                                                                     skip, limit, keyspace_only);
  if (hashes.empty()) {
    // The stdout pipeline.  The GPU contexts are created (and their stream buffers made)
    // on a second thread while this one reads the first batch, which is small so output
    // starts early; two contexts on two threads then take alternate batches and write
    // them in batch order.
    a5x_ctx* cx[2] = {nullptr, nullptr};
    int irc[2] = {0, 0};
    std::string ierr[2];
    auto make_ctx = [&](int i) {
      irc[i] = a5x_create(device, &cx[i]);
      if (irc[i]) {
        char m[96];
        snprintf(m, sizeof m, "a5_generator: no usable GPU (a5x_create=%d)", irc[i]);
        ierr[i] = m;
        return;
      }
      for (size_t t = 0; irc[i] == 0 && t < tables.size(); t++) {
        irc[i] = a5x_load_table_file(cx[i], tables[t].c_str());
        if (irc[i]) ierr[i] = a5x_last_error(cx[i]);  // log.Fatal (main.go:43-45)
      }
      if (irc[i] == 0) (void)a5x_stream_reserve(cx[i], B, BB);  // (optional warm-up)
      TL("context %d ready", i + 1);
    };
    std::thread init0(make_ctx, 0), init1(make_ctx, 1);
    // the first two batches (the first one small, so output starts early) are read while
    // the runtime and the contexts come up
    FILE* f = fopen(dict.c_str(), "rb");
    DictStream ds(f, chunk);
    std::vector<uint8_t> pw[2];
    std::vector<uint64_t> po[2];
    int npre = 0;
    if (f && ds.next(pw[0], po[0], std::max<uint64_t>(1, B / 16), BB / 16)) npre = 1;
    if (npre == 1 && ds.next(pw[1], po[1], B, BB)) npre = 2;
    TL("first batches read (%d)", npre);
    init0.join();
    init1.join();
    for (int i = 0; i < 2; i++)
      if (irc[i]) {  // the tables are read before the dictionary is opened (main.go:40-56)
        fprintf(stderr, "%s\n", ierr[i].c_str());
        if (f) fclose(f);
        return 1;
      }
    if (!f) { perror(dict.c_str()); return 1; }
    int rc = 0;
    Turn turn;
    std::mutex qmu;
    std::condition_variable qcv;
    std::deque<std::pair<uint64_t, std::pair<std::vector<uint8_t>, std::vector<uint64_t>>>> q[2];
    bool done_reading = false;
    std::atomic<int> failed{0};  // first error code (later batches are skipped)
    std::string emsg;
    auto worker = [&](int w) {
      for (;;) {
        std::pair<uint64_t, std::pair<std::vector<uint8_t>, std::vector<uint64_t>>> job;
        {
          std::unique_lock<std::mutex> l(qmu);
          qcv.wait(l, [&] { return !q[w].empty() || done_reading; });
          if (q[w].empty()) return;
          job = std::move(q[w].front());
          q[w].pop_front();
          qcv.notify_all();
        }
        const uint64_t k = job.first;
        auto& words = job.second.first;
        auto& off = job.second.second;
        SinkCtx sc{&turn, k, false, &failed, 0};
        TL("batch %llu: ctx %d starts (%zu words)", (unsigned long long)k, w, off.size() - 1);
        int r = failed.load() ? 0 : a5x_expand(cx[w], words.data(), off.data(), off.size() - 1, mode, tmin,
                                               tmax, sink_ordered, &sc, nullptr);
        if (!sc.waited) turn.wait(k);  // (a batch with no output still takes its turn)
        if (r == A5X_E_SINK && failed.load()) r = 0;  // stopped by an earlier batch's failure
        TL("batch %llu: done, %llu bytes", (unsigned long long)k, (unsigned long long)sc.bytes);
        int zero = 0;
        if (r && failed.compare_exchange_strong(zero, r)) emsg = a5x_last_error(cx[w]);
        turn.done(k);
      }
    };
    std::thread th0(worker, 0), th1(worker, 1);
    for (uint64_t k = 0;; k++) {
      std::vector<uint8_t> words;
      std::vector<uint64_t> off;
      if (k < 2) {
        if ((int)k >= npre) break;
        words.swap(pw[k]);
        off.swap(po[k]);
      } else {
        words.reserve(BB + 16 + (1 << 16));
        off.reserve(std::min<uint64_t>(B, 1u << 24) + 1);
        if (!ds.next(words, off, B, BB)) break;
        TL("batch %llu read (%zu words)", (unsigned long long)k, off.size() - 1);
      }
      std::unique_lock<std::mutex> l(qmu);
      qcv.wait(l, [&] { return q[k & 1].empty() || failed.load(); });  // one batch ahead per context
      if (failed.load()) break;
      q[k & 1].emplace_back(k, std::make_pair(std::move(words), std::move(off)));
      qcv.notify_all();
    }
    {
      std::lock_guard<std::mutex> l(qmu);
      done_reading = true;
      qcv.notify_all();
    }
    th0.join();
    th1.join();
    rc = failed.load();
    fclose(f);
    if (fflush(stdout) != 0 || ferror(stdout)) {  // (ENOSPC / EPIPE on the last buffer: not a success)
      if (!rc) emsg = std::string("writing stdout: ") + strerror(errno);
      rc = 1;
    }
    TL("all batches written");
    if (rc) fprintf(stderr, "a5_generator: %s\n", emsg.c_str());
    fflush(stderr);
    // (every device call has completed; the process's GPU state goes with it -- tearing
    // the two contexts down first only costs time)
    _exit(rc ? 2 : 0);
  }
  a5x_ctx* ctx = nullptr;
  int rc = a5x_create(device, &ctx);
  TL("context 1 created");
  if (rc) { fprintf(stderr, "a5_generator: no usable GPU (a5x_create=%d)\n", rc); return 1; }
  for (auto& t : tables) {
    rc = a5x_load_table_file(ctx, t.c_str());
    if (rc) { fprintf(stderr, "%s\n", a5x_last_error(ctx)); a5x_destroy(ctx); return 1; }  // log.Fatal
  }
  FILE* f = fopen(dict.c_str(), "rb");
  if (!f) { perror(dict.c_str()); a5x_destroy(ctx); return 1; }
  if ((rc = load_targets(ctx, hashes.c_str(), algo))) {
    fprintf(stderr, "a5_generator: %s\n", rc == A5X_E_IO ? "cannot read --hashes file" : a5x_last_error(ctx));
    a5x_destroy(ctx);
    fclose(f);
    return 1;
  }
  DictStream ds(f, chunk);
  std::vector<uint8_t> words;
  std::vector<uint64_t> sub;
  std::vector<a5x_hit> hits(1 << 16);
  std::unordered_set<std::string> cracked;  // each target reported once (hashcat potfile)
  while (rc == 0 && ds.next(words, sub, B, BB)) {
    const uint64_t nb = sub.size() - 1;
    const uint8_t* wb = words.data();
    uint64_t nh = 0;
    rc = a5x_expand_digest(ctx, wb, sub.data(), nb, mode, tmin, tmax, hits.data(), hits.size(), &nh, nullptr);
    if (rc == A5X_E_CAPACITY && nh > hits.size()) {
      hits.resize(nh);
      rc = a5x_expand_digest(ctx, wb, sub.data(), nb, mode, tmin, tmax, hits.data(), hits.size(), &nh, nullptr);
    }
    if (rc) break;
    // stream order, then the first candidate of each digest
    std::sort(hits.begin(), hits.begin() + nh, [](const a5x_hit& x, const a5x_hit& y) {
      return x.word != y.word ? x.word < y.word : x.cand < y.cand;
    });
    std::vector<a5x_hit> first;
    for (uint64_t h = 0; h < nh; h++)
      if (cracked.insert(std::string((const char*)hits[h].digest, 16)).second) first.push_back(hits[h]);
    rc = a5x_format_hits(ctx, wb, sub.data(), nb, mode, tmin, tmax, first.data(), first.size(), sink_stdout,
                         nullptr);
  }
  fclose(f);
  fflush(stdout);
  if (rc) fprintf(stderr, "a5_generator: %s\n", a5x_last_error(ctx));
  a5x_destroy(ctx);
  return rc ? 2 : 0;
}
