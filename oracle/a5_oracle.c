/*
 * a5_oracle.c -- CPU restatement of the reference main.go. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this
 * library (oracle/_build/liba5oracle.so); the product (liba5x.so) never links it.
 *
 * Restates /root/reference/main.go (go 1.23.5, go.mod:3):
 *   readSubstitutionTable      main.go:108-144   -> a5o_table_parse()
 *   decodeHexNotation          main.go:147-162   -> decode_hex_notation()
 *   -t merge                   main.go:40-50     -> a5o_table_load_file() in call order
 *   processWord                main.go:168-205   -> eng_default()
 *   processWordReverse (+bug)  main.go:208-305   -> eng_reverse()
 *   processWordSubstituteAll   main.go:308-365   -> eng_suball()  (sorted-order application)
 *   ...SubstituteAllReverse    main.go:369-440   -> eng_suball_rev()
 *   writer/channel/semaphore   main.go:58-98     -> a5o_run_pipeline()
 * Go stdlib semantics (bufio.ScanLines, strings.TrimSpace, hex.DecodeString,
 * strings.ReplaceAll) follow SURVEY.md Appendix A; oracle/a5_oracle.py is the
 * line-for-line Python twin and both are pinned by tests/golden.
 *
 * One deliberate speed-only difference: the default/-r engines skip map lookups
 * of substrings longer than the longest key (a Go map lookup of such a string
 * always misses), so the CPU baseline is, if anything, faster than the reference.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <sched.h>
#include <time.h>
#include <stdatomic.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#define A5O_EXPORT __attribute__((visibility("default")))

enum { MODE_DEFAULT = 0, MODE_REVERSE = 1, MODE_SUBALL = 2, MODE_SUBALL_REV = 3 };
enum { A5O_OK = 0, A5O_E_IO = -1, A5O_E_TOOLONG = -2, A5O_E_PANIC = -3, A5O_E_NOMEM = -4,
       A5O_E_ARG = -5 };

/* ------------------------------------------------------------------------ */
/* byte strings and the substitution map (Go map[string][]string)           */
/* ------------------------------------------------------------------------ */
typedef struct { uint8_t *p; size_t n; } bstr;

typedef struct {
    bstr key;
    bstr *vals;
    size_t nvals, cap;
} entry;

typedef struct a5o_table {
    entry *ents;        /* insertion order */
    size_t nents, cap;
    int64_t *slots;     /* open addressing: index into ents or -1 */
    size_t nslots;
    size_t maxklen;
} a5o_table;

static uint64_t fnv1a(const uint8_t *p, size_t n) {
    uint64_t h = 1469598103934665603ULL;
    for (size_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ULL; }
    return h;
}

static uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

/* Candidate hash of the multiset digest: fmix64(fnv1a64(bytes)).  The GPU
 * digest kernel (hashcat_a5_table_generator_amd/csrc/a5x_kernels.hip) uses the
 * same definition. */
A5O_EXPORT uint64_t a5o_cand_hash(const uint8_t *p, size_t n) { return fmix64(fnv1a(p, n)); }

static void *xrealloc(void *p, size_t n) {
    void *q = realloc(p, n ? n : 1);
    if (!q) { fprintf(stderr, "a5_oracle: out of memory\n"); abort(); }
    return q;
}

static bstr bdup(const uint8_t *p, size_t n) {
    bstr b; b.p = (uint8_t *)xrealloc(NULL, n + 1); if (n) memcpy(b.p, p, n); b.p[n] = 0; b.n = n;
    return b;
}

static void rehash(a5o_table *t) {
    size_t ns = t->nslots ? t->nslots * 2 : 64;
    while (ns < t->nents * 2 + 2) ns *= 2;
    free(t->slots);
    t->slots = (int64_t *)xrealloc(NULL, ns * sizeof(int64_t));
    for (size_t i = 0; i < ns; i++) t->slots[i] = -1;
    t->nslots = ns;
    for (size_t e = 0; e < t->nents; e++) {
        size_t h = fnv1a(t->ents[e].key.p, t->ents[e].key.n) & (ns - 1);
        while (t->slots[h] >= 0) h = (h + 1) & (ns - 1);
        t->slots[h] = (int64_t)e;
    }
}

static const entry *lookup(const a5o_table *t, const uint8_t *p, size_t n) {
    if (!t->nslots) return NULL;
    size_t h = fnv1a(p, n) & (t->nslots - 1);
    for (;;) {
        int64_t e = t->slots[h];
        if (e < 0) return NULL;
        const entry *en = &t->ents[e];
        if (en->key.n == n && (n == 0 || memcmp(en->key.p, p, n) == 0)) return en;
        h = (h + 1) & (t->nslots - 1);
    }
}

A5O_EXPORT a5o_table *a5o_table_new(void) { return (a5o_table *)calloc(1, sizeof(a5o_table)); }

A5O_EXPORT void a5o_table_free(a5o_table *t) {
    if (!t) return;
    for (size_t e = 0; e < t->nents; e++) {
        free(t->ents[e].key.p);
        for (size_t v = 0; v < t->ents[e].nvals; v++) free(t->ents[e].vals[v].p);
        free(t->ents[e].vals);
    }
    free(t->ents); free(t->slots); free(t);
}

/* substitutionMap[key] = append(substitutionMap[key], value)  (main.go:141, 48) */
A5O_EXPORT int a5o_table_add(a5o_table *t, const uint8_t *k, size_t kn, const uint8_t *v, size_t vn) {
    entry *en = (entry *)lookup(t, k, kn);
    if (!en) {
        if (t->nents == t->cap) {
            t->cap = t->cap ? t->cap * 2 : 16;
            t->ents = (entry *)xrealloc(t->ents, t->cap * sizeof(entry));
        }
        en = &t->ents[t->nents++];
        memset(en, 0, sizeof(*en));
        en->key = bdup(k, kn);
        if (kn > t->maxklen) t->maxklen = kn;
        if (t->nents * 2 + 2 > t->nslots) rehash(t);
        else {
            size_t h = fnv1a(k, kn) & (t->nslots - 1);
            while (t->slots[h] >= 0) h = (h + 1) & (t->nslots - 1);
            t->slots[h] = (int64_t)(t->nents - 1);
        }
        en = (entry *)lookup(t, k, kn);
    }
    if (en->nvals == en->cap) {
        en->cap = en->cap ? en->cap * 2 : 2;
        en->vals = (bstr *)xrealloc(en->vals, en->cap * sizeof(bstr));
    }
    en->vals[en->nvals++] = bdup(v, vn);
    return A5O_OK;
}

A5O_EXPORT size_t a5o_table_nkeys(const a5o_table *t) { return t->nents; }

/* ------------------------------------------------------------------------ */
/* Go stdlib restatements                                                    */
/* ------------------------------------------------------------------------ */
#define RUNE_ERROR 0xFFFD

static int decode_rune(const uint8_t *s, size_t n, int *size) {
    if (n == 0) { *size = 0; return RUNE_ERROR; }
    uint8_t b0 = s[0];
    if (b0 < 0x80) { *size = 1; return b0; }
    int sz; uint8_t lo = 0x80, hi = 0xBF;
    if (b0 >= 0xC2 && b0 <= 0xDF) sz = 2;
    else if (b0 >= 0xE0 && b0 <= 0xEF) { sz = 3; if (b0 == 0xE0) lo = 0xA0; if (b0 == 0xED) hi = 0x9F; }
    else if (b0 >= 0xF0 && b0 <= 0xF4) { sz = 4; if (b0 == 0xF0) lo = 0x90; if (b0 == 0xF4) hi = 0x8F; }
    else { *size = 1; return RUNE_ERROR; }
    if (n < (size_t)sz || s[1] < lo || s[1] > hi) { *size = 1; return RUNE_ERROR; }
    for (int k = 2; k < sz; k++)
        if (s[k] < 0x80 || s[k] > 0xBF) { *size = 1; return RUNE_ERROR; }
    *size = sz;
    if (sz == 2) return ((b0 & 0x1F) << 6) | (s[1] & 0x3F);
    if (sz == 3) return ((b0 & 0x0F) << 12) | ((s[1] & 0x3F) << 6) | (s[2] & 0x3F);
    return ((b0 & 0x07) << 18) | ((s[1] & 0x3F) << 12) | ((s[2] & 0x3F) << 6) | (s[3] & 0x3F);
}

static int decode_last_rune(const uint8_t *s, size_t end, int *size) {
    if (end == 0) { *size = 0; return RUNE_ERROR; }
    ptrdiff_t start = (ptrdiff_t)end - 1;
    if (s[start] < 0x80) { *size = 1; return s[start]; }
    ptrdiff_t lim = (ptrdiff_t)end - 4; if (lim < 0) lim = 0;
    for (start--; start >= lim; start--) if ((s[start] & 0xC0) != 0x80) break;
    if (start < 0) start = 0;
    int sz; int r = decode_rune(s + start, end - (size_t)start, &sz);
    if ((size_t)start + (size_t)sz != end) { *size = 1; return RUNE_ERROR; }
    *size = sz; return r;
}

static int is_unicode_space(int r) {
    switch (r) {
    case 0x09: case 0x0A: case 0x0B: case 0x0C: case 0x0D: case 0x20: case 0x85: case 0xA0:
    case 0x1680: case 0x2028: case 0x2029: case 0x202F: case 0x205F: case 0x3000: return 1;
    default: return r >= 0x2000 && r <= 0x200A;
    }
}

static int is_ascii_space(uint8_t c) {
    return c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r' || c == ' ';
}

static void trim_right_func(const uint8_t *s, size_t *len) {
    size_t end = *len;
    while (end > 0) {
        int sz; int r = decode_last_rune(s, end, &sz);
        if (!is_unicode_space(r)) break;
        end -= (size_t)sz;
    }
    *len = end;
}

/* strings.TrimSpace (go1.23 strings.go): returns [*b, *b+*n) */
static void trim_space(const uint8_t **b, size_t *n) {
    const uint8_t *s = *b; size_t len = *n, start = 0;
    for (; start < len; start++) {
        uint8_t c = s[start];
        if (c >= 0x80) {  /* TrimFunc(s[start:], unicode.IsSpace) */
            const uint8_t *p = s + start; size_t m = len - start, i = 0;
            while (i < m) { int sz; int r = decode_rune(p + i, m - i, &sz); if (!is_unicode_space(r)) break; i += (size_t)sz; }
            p += i; m -= i;
            trim_right_func(p, &m);
            *b = p; *n = m; return;
        }
        if (!is_ascii_space(c)) break;
    }
    size_t stop = len;
    for (; stop > start; stop--) {
        uint8_t c = s[stop - 1];
        if (c >= 0x80) {
            size_t m = stop - start; trim_right_func(s + start, &m);
            *b = s + start; *n = m; return;
        }
        if (!is_ascii_space(c)) break;
    }
    *b = s + start; *n = stop - start;
}

static int hexval(uint8_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

/* decodeHexNotation (main.go:147-162). out must hold n bytes. returns -1 on error. */
static long decode_hex_notation(const uint8_t *v, size_t n, uint8_t *out) {
    if (n < 7 || memcmp(v, "$HEX[", 5) != 0 || v[n - 1] != ']') { memcpy(out, v, n); return (long)n; }
    uint8_t tmp[n]; size_t m = 0;
    for (size_t i = 5; i + 1 < n; i++) if (v[i] != ' ') tmp[m++] = v[i];
    if (m % 2) return -1;
    for (size_t i = 0; i < m; i += 2) {
        int a = hexval(tmp[i]), b = hexval(tmp[i + 1]);
        if (a < 0 || b < 0) return -1;
        out[i / 2] = (uint8_t)((a << 4) | b);
    }
    return (long)(m / 2);
}

#define SCAN_MAX (64 * 1024)

/* bufio.Scanner+ScanLines: next line in [*pos, n). returns 1 token, 0 end, -1 ErrTooLong */
static int scan_line(const uint8_t *d, size_t n, size_t *pos, const uint8_t **line, size_t *len) {
    if (*pos >= n) return 0;
    size_t lim = n - *pos; if (lim > SCAN_MAX) lim = SCAN_MAX;
    const uint8_t *nl = (const uint8_t *)memchr(d + *pos, '\n', lim);
    size_t l;
    if (!nl) {
        if (n - *pos >= SCAN_MAX) return -1;
        l = n - *pos; *line = d + *pos; *pos = n;
    } else {
        l = (size_t)(nl - (d + *pos)); *line = d + *pos; *pos += l + 1;
    }
    if (l && (*line)[l - 1] == '\r') l--;
    *len = l;
    return 1;
}

/* readSubstitutionTable on file bytes, merged into t (main.go:108-144, 40-50).
 * Because merge is append-per-key in -t order, parsing file after file
 * straight into the merged map yields the same value order. */
A5O_EXPORT int a5o_table_parse(a5o_table *t, const uint8_t *d, size_t n) {
    size_t pos = 0; const uint8_t *line; size_t len; int r;
    /* per-file map first: keys new to this file are appended in one go at the
     * end of the file exactly like main.go:47-49 appends values... per key */
    a5o_table *ft = a5o_table_new();
    while ((r = scan_line(d, n, &pos, &line, &len)) == 1) {
        const uint8_t *s = line; size_t m = len;
        trim_space(&s, &m);
        if (m == 0 || s[0] == '#') continue;
        const uint8_t *eq = (const uint8_t *)memchr(s, '=', m);
        if (!eq) continue;
        size_t kn = (size_t)(eq - s), vn = m - kn - 1;
        uint8_t kb[kn + 1], vb[vn + 1];
        long kd = decode_hex_notation(s, kn, kb);
        if (kd < 0) { fprintf(stderr, "Error decoding hex notation in key: %.*s\n", (int)m, s); continue; }
        long vd = decode_hex_notation(eq + 1, vn, vb);
        if (vd < 0) { fprintf(stderr, "Error decoding hex notation in value: %.*s\n", (int)m, s); continue; }
        a5o_table_add(ft, kb, (size_t)kd, vb, (size_t)vd);
    }
    if (r < 0) { a5o_table_free(ft); return A5O_E_TOOLONG; }
    for (size_t e = 0; e < ft->nents; e++)
        for (size_t v = 0; v < ft->ents[e].nvals; v++)
            a5o_table_add(t, ft->ents[e].key.p, ft->ents[e].key.n, ft->ents[e].vals[v].p, ft->ents[e].vals[v].n);
    a5o_table_free(ft);
    return A5O_OK;
}

A5O_EXPORT int a5o_table_load_file(a5o_table *t, const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) return A5O_E_IO;
    size_t cap = 1 << 16, n = 0; uint8_t *d = (uint8_t *)xrealloc(NULL, cap);
    size_t r;
    while ((r = fread(d + n, 1, cap - n, f)) > 0) { n += r; if (n == cap) { cap *= 2; d = (uint8_t *)xrealloc(d, cap); } }
    fclose(f);
    int rc = a5o_table_parse(t, d, n);
    free(d);
    return rc;
}

/* Export the merged map (keys in first-appearance order) for cross-checking the
 * product parser.  Layout: keys/values as concatenated bytes with offsets. */
A5O_EXPORT size_t a5o_table_nvals(const a5o_table *t) {
    size_t s = 0; for (size_t e = 0; e < t->nents; e++) s += t->ents[e].nvals; return s;
}
A5O_EXPORT int a5o_table_get(const a5o_table *t, size_t e, const uint8_t **key, size_t *klen, size_t *nvals) {
    if (e >= t->nents) return A5O_E_ARG;
    *key = t->ents[e].key.p; *klen = t->ents[e].key.n; *nvals = t->ents[e].nvals; return A5O_OK;
}
A5O_EXPORT int a5o_table_get_val(const a5o_table *t, size_t e, size_t v, const uint8_t **val, size_t *vlen) {
    if (e >= t->nents || v >= t->ents[e].nvals) return A5O_E_ARG;
    *val = t->ents[e].vals[v].p; *vlen = t->ents[e].vals[v].n; return A5O_OK;
}

/* ------------------------------------------------------------------------ */
/* Engines                                                                   */
/* ------------------------------------------------------------------------ */
typedef void (*a5o_emit_fn)(void *user, const uint8_t *s, size_t n);

typedef struct { uint8_t *p; size_t n, cap; } buf;
static void buf_reserve(buf *b, size_t n) { if (n > b->cap) { b->cap = n * 2; b->p = (uint8_t *)xrealloc(b->p, b->cap); } }

/* processWord (main.go:168-205). cur = current word bytes; start in cur coords. */
typedef struct { const a5o_table *t; int mn, mx; a5o_emit_fn emit; void *user; } dctx;

static void gen_default(dctx *c, const uint8_t *cur, size_t n, int cnt, size_t start) {
    for (size_t i = start; i < n; i++) {
        size_t kmax = n - i; if (kmax > c->t->maxklen) kmax = c->t->maxklen;
        for (size_t kl = kmax; kl >= 1; kl--) {
            const entry *en = lookup(c->t, cur + i, kl);
            if (!en) continue;
            for (size_t v = 0; v < en->nvals; v++) {
                const bstr *s = &en->vals[v];
                int nc = cnt + 1;
                if (nc > c->mx) continue;
                size_t nn = i + s->n + (n - i - kl);
                uint8_t *nw = (uint8_t *)xrealloc(NULL, nn + 1);
                memcpy(nw, cur, i); memcpy(nw + i, s->p, s->n); memcpy(nw + i + s->n, cur + i + kl, n - i - kl);
                if (nc >= c->mn) c->emit(c->user, nw, nn);
                gen_default(c, nw, nn, nc, i + s->n);
                free(nw);
            }
        }
    }
}

static int eng_default(const a5o_table *t, const uint8_t *w, size_t n, int mn, int mx, a5o_emit_fn emit, void *user) {
    if (mn == 0) mn = 1;
    dctx c = { t, mn, mx, emit, user };
    gen_default(&c, w, n, 0, 0);
    return A5O_OK;
}

/* processWordReverse (main.go:208-261) with generateCombinations (263-281),
 * validSubstitutionPositions (283-305) and the running-offset bug. */
typedef struct { size_t start, kl; const entry *en; } rpos;

static int rev_apply(const uint8_t *w, size_t n, const rpos *pos, const int *combo, int k,
                     a5o_emit_fn emit, void *user, buf *tmp, buf *tmp2) {
    /* validity: sort intervals by start, reject overlaps */
    for (int a = 0; a < k; a++)
        for (int b = 0; b < k; b++) {
            if (a == b) continue;
            const rpos *x = &pos[combo[a]], *y = &pos[combo[b]];
            /* overlap of closed intervals [s, s+kl-1] */
            if (x->start <= y->start && y->start <= x->start + x->kl - 1) return 0;
        }
    buf_reserve(tmp, n + 1); memcpy(tmp->p, w, n); tmp->n = n;
    long off = 0;
    for (int a = 0; a < k; a++) {
        const rpos *p = &pos[combo[a]];
        const bstr *s0 = &p->en->vals[0];
        long st = (long)p->start + off, en = st + (long)p->kl;
        if (st < 0 || en > (long)tmp->n) return A5O_E_PANIC;
        size_t nn = (size_t)st + s0->n + (tmp->n - (size_t)en);
        buf_reserve(tmp2, nn + 1);
        memcpy(tmp2->p, tmp->p, (size_t)st); memcpy(tmp2->p + st, s0->p, s0->n);
        memcpy(tmp2->p + st + s0->n, tmp->p + en, tmp->n - (size_t)en);
        tmp2->n = nn;
        buf t3 = *tmp; *tmp = *tmp2; *tmp2 = t3;
        off += (long)s0->n - (long)p->kl;
    }
    emit(user, tmp->p, tmp->n);
    return 0;
}

/* enumerate combos of k out of n with indices descending, in Go's order */
static int rev_combos(const uint8_t *w, size_t wn, const rpos *pos, int n, int k, int *combo, int depth,
                      a5o_emit_fn emit, void *user, buf *t1, buf *t2) {
    if (depth == k) return rev_apply(w, wn, pos, combo, k, emit, user, t1, t2);
    int hi = depth == 0 ? n - 1 : combo[depth - 1] - 1;
    for (int i = hi; i >= k - depth - 1; i--) {
        combo[depth] = i;
        int r = rev_combos(w, wn, pos, n, k, combo, depth + 1, emit, user, t1, t2);
        if (r) return r;
    }
    return 0;
}

static int eng_reverse(const a5o_table *t, const uint8_t *w, size_t n, int mn, int mx, a5o_emit_fn emit, void *user) {
    size_t cap = 16, np = 0; rpos *pos = (rpos *)xrealloc(NULL, cap * sizeof(rpos));
    for (size_t i = 0; i < n; i++)
        for (size_t kl = 1; kl <= n - i && kl <= t->maxklen; kl++) {
            const entry *en = lookup(t, w + i, kl);
            if (!en) continue;
            if (np == cap) { cap *= 2; pos = (rpos *)xrealloc(pos, cap * sizeof(rpos)); }
            pos[np].start = i; pos[np].kl = kl; pos[np].en = en; np++;
        }
    int total = (int)np, rc = 0;
    if (total < mn) { free(pos); return 0; }
    int amax = mx < total ? mx : total;
    if (mn < 0 && amax >= mn) { free(pos); return A5O_E_PANIC; } /* Go: unbounded recursion (k<0) */
    int *combo = (int *)xrealloc(NULL, (size_t)(total + 1) * sizeof(int));
    buf t1 = {0}, t2 = {0};
    for (int k = amax; k >= mn && !rc; k--) rc = rev_combos(w, n, pos, total, k, combo, 0, emit, user, &t1, &t2);
    free(combo); free(pos); free(t1.p); free(t2.p);
    return rc;
}

/* -s helpers: unique patterns present (main.go:310-326), sorted bytewise */
static int bstr_cmp(const void *a, const void *b) {
    const entry *x = *(const entry *const *)a, *y = *(const entry *const *)b;
    size_t m = x->key.n < y->key.n ? x->key.n : y->key.n;
    int c = m ? memcmp(x->key.p, y->key.p, m) : 0;
    if (c) return c;
    return (x->key.n > y->key.n) - (x->key.n < y->key.n);
}

static size_t find_patterns(const a5o_table *t, const uint8_t *w, size_t n, const entry ***out) {
    const entry **p = (const entry **)xrealloc(NULL, (t->nents + 1) * sizeof(entry *));
    size_t np = 0;
    if (n > 0)
        for (size_t e = 0; e < t->nents; e++) {
            const bstr *k = &t->ents[e].key;
            int found = 0;
            if (k->n == 0) found = 1;
            else if (k->n <= n)
                for (size_t i = 0; i + k->n <= n && !found; i++) found = memcmp(w + i, k->p, k->n) == 0;
            if (found) p[np++] = &t->ents[e];
        }
    qsort(p, np, sizeof(entry *), bstr_cmp);
    *out = p;
    return np;
}

/* strings.ReplaceAll(src, old, new) into dst */
static void replace_all(buf *dst, const uint8_t *s, size_t n, const bstr *old, const bstr *nw) {
    dst->n = 0;
    if (old->n == 0) {
        size_t i = 0;
        buf_reserve(dst, nw->n * (n + 1) + n + 1);
        memcpy(dst->p, nw->p, nw->n); dst->n = nw->n;
        while (i < n) {
            int sz; decode_rune(s + i, n - i, &sz);
            memcpy(dst->p + dst->n, s + i, (size_t)sz); dst->n += (size_t)sz;
            memcpy(dst->p + dst->n, nw->p, nw->n); dst->n += nw->n;
            i += (size_t)sz;
        }
        return;
    }
    size_t i = 0;
    buf_reserve(dst, n + 1);
    while (i < n) {
        const uint8_t *hit = NULL;
        if (i + old->n <= n) hit = (const uint8_t *)memmem(s + i, n - i, old->p, old->n);
        if (!hit) { buf_reserve(dst, dst->n + (n - i) + 1); memcpy(dst->p + dst->n, s + i, n - i); dst->n += n - i; break; }
        size_t h = (size_t)(hit - s);
        buf_reserve(dst, dst->n + (h - i) + nw->n + 1);
        memcpy(dst->p + dst->n, s + i, h - i); dst->n += h - i;
        memcpy(dst->p + dst->n, nw->p, nw->n); dst->n += nw->n;
        i = h + old->n;
    }
}

typedef struct {
    const uint8_t *w; size_t n; const entry **pats; size_t np; int mn, mx;
    const bstr **choice;  /* per pattern: NULL = not substituted */
    a5o_emit_fn emit; void *user; buf a, b;
} sctx;

static void suball_leaf(sctx *c, size_t cnt) {
    if ((long)cnt < c->mn || (long)cnt > c->mx) return;
    buf_reserve(&c->a, c->n + 1); memcpy(c->a.p, c->w, c->n); c->a.n = c->n;
    for (size_t i = 0; i < c->np; i++) {       /* canonical: sorted pattern order */
        if (!c->choice[i]) continue;
        replace_all(&c->b, c->a.p, c->a.n, &c->pats[i]->key, c->choice[i]);
        buf t = c->a; c->a = c->b; c->b = t;
    }
    c->emit(c->user, c->a.p, c->a.n);
}

static void gen_suball(sctx *c, size_t pos, size_t cnt) {
    if (pos >= c->np) { suball_leaf(c, cnt); return; }
    const entry *p = c->pats[pos];
    for (size_t v = 0; v < p->nvals; v++) { c->choice[pos] = &p->vals[v]; gen_suball(c, pos + 1, cnt + 1); }
    c->choice[pos] = NULL;
    gen_suball(c, pos + 1, cnt);
}

static int eng_suball(const a5o_table *t, const uint8_t *w, size_t n, int mn, int mx, a5o_emit_fn emit, void *user) {
    sctx c; memset(&c, 0, sizeof(c));
    c.w = w; c.n = n; c.mn = mn; c.mx = mx; c.emit = emit; c.user = user;
    c.np = find_patterns(t, w, n, &c.pats);
    c.choice = (const bstr **)calloc(c.np + 1, sizeof(bstr *));
    gen_suball(&c, 0, 0);
    free(c.choice); free(c.pats); free(c.a.p); free(c.b.p);
    return A5O_OK;
}

static void gen_suball_rev(sctx *c, size_t pos, size_t cnt) {
    if ((long)cnt < c->mn) return;
    if ((long)cnt <= c->mx) {
        long save = c->mn; c->mn = -2147483647; suball_leaf(c, cnt); c->mn = (int)save;
    }
    if ((long)cnt <= c->mn) return;
    for (size_t i = pos; i < c->np; i++) {
        if (!c->choice[i]) continue;
        const bstr *keep = c->choice[i];
        c->choice[i] = NULL;
        gen_suball_rev(c, i + 1, cnt - 1);
        c->choice[i] = keep;
    }
}

static int eng_suball_rev(const a5o_table *t, const uint8_t *w, size_t n, int mn, int mx, a5o_emit_fn emit, void *user) {
    sctx c; memset(&c, 0, sizeof(c));
    c.w = w; c.n = n; c.mn = mn; c.mx = mx; c.emit = emit; c.user = user;
    c.np = find_patterns(t, w, n, &c.pats);
    if ((long)c.np < mn) { free(c.pats); return A5O_OK; }
    c.choice = (const bstr **)calloc(c.np + 1, sizeof(bstr *));
    for (size_t i = 0; i < c.np; i++) c.choice[i] = &c.pats[i]->vals[0];
    gen_suball_rev(&c, 0, c.np);
    free(c.choice); free(c.pats); free(c.a.p); free(c.b.p);
    return A5O_OK;
}

A5O_EXPORT int a5o_expand_word(const a5o_table *t, const uint8_t *w, size_t n, int mode, int mn, int mx,
                               a5o_emit_fn emit, void *user) {
    switch (mode) {
    case MODE_DEFAULT: return eng_default(t, w, n, mn, mx, emit, user);
    case MODE_REVERSE: return eng_reverse(t, w, n, mn, mx, emit, user);
    case MODE_SUBALL: return eng_suball(t, w, n, mn, mx, emit, user);
    case MODE_SUBALL_REV: return eng_suball_rev(t, w, n, mn, mx, emit, user);
    default: return A5O_E_ARG;
    }
}

/* ------------------------------------------------------------------------ */
/* Batch helpers used by the parity tests                                    */
/* ------------------------------------------------------------------------ */
typedef struct { uint64_t cnt, bytes, hsum, hsq; } digest;

static void emit_digest(void *u, const uint8_t *s, size_t n) {
    digest *d = (digest *)u;
    uint64_t h = a5o_cand_hash(s, n);
    d->cnt++; d->bytes += n + 1; d->hsum += h; d->hsq += h * h;
}

typedef struct {
    const a5o_table *t; const uint8_t *words; const uint64_t *off; size_t nw;
    int mode, mn, mx; uint64_t *out; atomic_size_t next; atomic_int err;
} digest_job;

static void *digest_worker(void *arg) {
    digest_job *j = (digest_job *)arg;
    for (;;) {
        size_t i = atomic_fetch_add(&j->next, 64);
        if (i >= j->nw) break;
        size_t e = i + 64 < j->nw ? i + 64 : j->nw;
        for (; i < e; i++) {
            digest d = {0, 0, 0, 0};
            int rc = a5o_expand_word(j->t, j->words + j->off[i], (size_t)(j->off[i + 1] - j->off[i]),
                                     j->mode, j->mn, j->mx, emit_digest, &d);
            if (rc) atomic_store(&j->err, rc);
            j->out[4 * i + 0] = d.cnt; j->out[4 * i + 1] = d.bytes;
            j->out[4 * i + 2] = d.hsum; j->out[4 * i + 3] = d.hsq;
        }
    }
    return NULL;
}

/* Per-word multiset digest {count, bytes incl '\n', sum h, sum h^2} (mod 2^64).
 * out has 4*nw u64.  words/off: concatenated words, off has nw+1 entries. */
A5O_EXPORT int a5o_digest_batch(const a5o_table *t, const uint8_t *words, const uint64_t *off, size_t nw,
                                int mode, int mn, int mx, uint64_t *out, int nthreads) {
    digest_job j; j.t = t; j.words = words; j.off = off; j.nw = nw; j.mode = mode; j.mn = mn; j.mx = mx;
    j.out = out; atomic_init(&j.next, 0); atomic_init(&j.err, 0);
    if (nthreads < 1) nthreads = 1;
    pthread_t th[256]; if (nthreads > 256) nthreads = 256;
    for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, digest_worker, &j);
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    return atomic_load(&j.err);
}

typedef struct { uint8_t *out; size_t cap, n; } collect;
static void emit_collect(void *u, const uint8_t *s, size_t n) {
    collect *c = (collect *)u;
    if (c->n + n + 1 <= c->cap) { memcpy(c->out + c->n, s, n); c->out[c->n + n] = '\n'; }
    c->n += n + 1;
}

/* Candidates of every word, "cand\n" in DFS order, words in order.  Returns the
 * byte count needed (written only if <= cap); negative = error code.
 * word_bytes (optional, nw entries) receives each word's output bytes. */
A5O_EXPORT int64_t a5o_expand_batch(const a5o_table *t, const uint8_t *words, const uint64_t *off, size_t nw,
                                    int mode, int mn, int mx, uint8_t *out, size_t cap, uint64_t *word_bytes) {
    collect c = { out, cap, 0 };
    for (size_t i = 0; i < nw; i++) {
        size_t before = c.n;
        int rc = a5o_expand_word(t, words + off[i], (size_t)(off[i + 1] - off[i]), mode, mn, mx, emit_collect, &c);
        if (rc) return rc;
        if (word_bytes) word_bytes[i] = c.n - before;
    }
    return (int64_t)c.n;
}

/* ------------------------------------------------------------------------ */
/* Reference-structured CPU pipeline (main.go:58-98): the CPU baseline.      */
/* nthreads workers (sem of size Threads, one word per task), a bounded      */
/* channel of capacity 1000 carrying one heap string per candidate, and one  */
/* writer goroutine with a 4 KiB bufio.Writer doing WriteString(s + "\n").   */
/* ------------------------------------------------------------------------ */
#define CHAN_CAP 1024  /* Go: make(chan string, 1000); a power of two for the ring index */
/* A buffered Go channel as a bounded lock-free MPMC ring (D. Vyukov's sequence-number
 * queue): a sender claims a slot with one CAS and publishes it with a release store;
 * the receiver takes slots in order.  A full (empty) channel makes the sender
 * (receiver) spin briefly and then PARK on a futex, like a goroutine parking on a
 * channel: it stops using a core (Go's scheduler runs something else), and it is
 * woken only when a receiver (sender) sees a parked waiter -- no syscall per message
 * while nobody sleeps.  (Round 1 used a mutex + condition variable per operation,
 * which serialised 16 senders on one futex; round 2's spin-then-yield kept every
 * blocked sender runnable, starving the writer whenever the host's CPU quota was
 * smaller than senders + 1.) */
/* A channel message: the candidate string and the worker whose pool it came from. */
typedef struct { bstr v; int owner; } chan_msg;
typedef struct { _Atomic size_t seq; chan_msg v; } chan_slot;
typedef struct {
    chan_slot q[CHAN_CAP];
    _Alignas(64) _Atomic size_t tail;  /* next slot to send into */
    _Alignas(64) _Atomic size_t head;  /* next slot to receive from (one receiver) */
    _Alignas(64) _Atomic int closed;
    _Alignas(64) _Atomic uint32_t hgen, swait;  /* receiver progress generation, parked senders */
    _Alignas(64) _Atomic uint32_t tgen, rwait;  /* sender progress generation, parked receiver */
} chan_t;

static void chan_init(chan_t *c) {
    for (size_t i = 0; i < CHAN_CAP; i++) atomic_init(&c->q[i].seq, i);
    atomic_init(&c->tail, 0); atomic_init(&c->head, 0); atomic_init(&c->closed, 0);
    atomic_init(&c->hgen, 0); atomic_init(&c->swait, 0); atomic_init(&c->tgen, 0); atomic_init(&c->rwait, 0);
}

static void futex_wait_u32(_Atomic uint32_t *a, uint32_t v) {  /* bounded park: a missed wake costs <= 50 us */
    struct timespec ts = {0, 50000};
    syscall(SYS_futex, (uint32_t *)a, FUTEX_WAIT_PRIVATE, v, &ts, NULL, 0);
}
static void futex_wake_all(_Atomic uint32_t *a) {
    syscall(SYS_futex, (uint32_t *)a, FUTEX_WAKE_PRIVATE, INT32_MAX, NULL, NULL, 0);
}

#define CHAN_SPIN 64

static void chan_send(chan_t *c, chan_msg s) {
    unsigned spins = 0;
    size_t pos = atomic_load_explicit(&c->tail, memory_order_relaxed);
    for (;;) {
        chan_slot *sl = &c->q[pos & (CHAN_CAP - 1)];
        const size_t seq = atomic_load_explicit(&sl->seq, memory_order_acquire);
        const intptr_t d = (intptr_t)seq - (intptr_t)pos;
        if (d == 0) {
            if (atomic_compare_exchange_weak_explicit(&c->tail, &pos, pos + 1, memory_order_relaxed,
                                                      memory_order_relaxed)) {
                sl->v = s;
                atomic_store_explicit(&sl->seq, pos + 1, memory_order_release);
                if (atomic_load_explicit(&c->rwait, memory_order_relaxed)) {  /* wake the parked receiver */
                    atomic_fetch_add_explicit(&c->tgen, 1, memory_order_relaxed);
                    futex_wake_all(&c->tgen);
                }
                return;
            }
        } else if (d < 0) {  /* full */
            if (++spins < CHAN_SPIN) {
                __builtin_ia32_pause();
            } else if (spins < CHAN_SPIN + 64) {
                sched_yield();
            } else {  /* park until the receiver frees a slot */
                const uint32_t g = atomic_load_explicit(&c->hgen, memory_order_relaxed);
                atomic_fetch_add_explicit(&c->swait, 1, memory_order_seq_cst);
                const size_t seq2 = atomic_load_explicit(&sl->seq, memory_order_acquire);
                if ((intptr_t)seq2 - (intptr_t)pos < 0) futex_wait_u32(&c->hgen, g);
                atomic_fetch_sub_explicit(&c->swait, 1, memory_order_relaxed);
                spins = 0;
            }
            pos = atomic_load_explicit(&c->tail, memory_order_relaxed);
        } else {
            pos = atomic_load_explicit(&c->tail, memory_order_relaxed);
        }
    }
}

static int chan_recv(chan_t *c, chan_msg *s) {
    unsigned spins = 0;
    const size_t pos = atomic_load_explicit(&c->head, memory_order_relaxed);
    chan_slot *sl = &c->q[pos & (CHAN_CAP - 1)];
    for (;;) {
        const size_t seq = atomic_load_explicit(&sl->seq, memory_order_acquire);
        if (seq == pos + 1) break;
        if (atomic_load_explicit(&c->closed, memory_order_acquire) &&
            atomic_load_explicit(&sl->seq, memory_order_acquire) != pos + 1)
            return 0;  /* closed after every sender finished: nothing left */
        if (++spins < CHAN_SPIN) {
            __builtin_ia32_pause();
        } else if (spins < CHAN_SPIN + 256) {
            sched_yield();  /* the writer stays runnable a while: senders are usually mid-word */
        } else {  /* park until a sender publishes (or the channel closes) */
            const uint32_t g = atomic_load_explicit(&c->tgen, memory_order_relaxed);
            atomic_store_explicit(&c->rwait, 1, memory_order_seq_cst);
            if (atomic_load_explicit(&sl->seq, memory_order_acquire) != pos + 1 &&
                !atomic_load_explicit(&c->closed, memory_order_acquire))
                futex_wait_u32(&c->tgen, g);
            atomic_store_explicit(&c->rwait, 0, memory_order_relaxed);
            spins = 0;
        }
    }
    *s = sl->v;
    atomic_store_explicit(&sl->seq, pos + CHAN_CAP, memory_order_release);
    atomic_store_explicit(&c->head, pos + 1, memory_order_relaxed);
    /* parked senders are woken together once the channel is half empty (one syscall
     * per ~CHAN_CAP/2 messages, like Go's cheap goready); parks are bounded, so no
     * fence is needed against a sender that parks concurrently */
    if (atomic_load_explicit(&c->swait, memory_order_relaxed) &&
        atomic_load_explicit(&c->tail, memory_order_relaxed) - (pos + 1) <= CHAN_CAP / 2) {
        atomic_fetch_add_explicit(&c->hgen, 1, memory_order_relaxed);
        futex_wake_all(&c->hgen);
    }
    return 1;
}

static void chan_close(chan_t *c) {
    atomic_store_explicit(&c->closed, 1, memory_order_seq_cst);
    atomic_fetch_add_explicit(&c->tgen, 1, memory_order_relaxed);
    futex_wake_all(&c->tgen);
}

/* Candidate strings come from per-worker pools of 128-B slots that the writer hands
 * back through a single-producer / single-consumer ring, like Go's per-P allocation
 * caches with the garbage collector reclaiming the writer's consumed strings: no
 * cross-thread malloc/free per candidate (glibc's arena locks made 16 workers slower
 * than one).  Longer strings use malloc. */
#define POOL_SLOT 128
#define POOL_RET 8192   /* return ring per worker (power of two) */
#define POOL_BLOCK (POOL_SLOT * 512)
typedef struct {
    uint8_t **ret;                      /* slots returned by the writer */
    _Alignas(64) _Atomic size_t rhead;  /* consumed by the worker */
    _Alignas(64) _Atomic size_t rtail;  /* produced by the writer */
    _Alignas(64) uint8_t *blk; size_t blk_used;
    uint8_t **blocks; size_t nblocks, cblocks;
} str_pool;

static uint8_t *pool_get(str_pool *P) {
    const size_t h = atomic_load_explicit(&P->rhead, memory_order_relaxed);
    if (h != atomic_load_explicit(&P->rtail, memory_order_acquire)) {
        uint8_t *x = P->ret[h & (POOL_RET - 1)];
        atomic_store_explicit(&P->rhead, h + 1, memory_order_release);
        return x;
    }
    if (!P->blk || P->blk_used == POOL_BLOCK) {
        if (P->nblocks == P->cblocks) {
            P->cblocks = P->cblocks ? 2 * P->cblocks : 64;
            P->blocks = (uint8_t **)xrealloc(P->blocks, P->cblocks * sizeof(uint8_t *));
        }
        P->blk = (uint8_t *)xrealloc(NULL, POOL_BLOCK);
        P->blocks[P->nblocks++] = P->blk;
        P->blk_used = 0;
    }
    uint8_t *x = P->blk + P->blk_used;
    P->blk_used += POOL_SLOT;
    return x;
}

static void pool_put(str_pool *P, uint8_t *x) {  /* writer side; a full ring keeps the slot */
    const size_t t = atomic_load_explicit(&P->rtail, memory_order_relaxed);
    if (t - atomic_load_explicit(&P->rhead, memory_order_acquire) >= POOL_RET) return;
    P->ret[t & (POOL_RET - 1)] = x;
    atomic_store_explicit(&P->rtail, t + 1, memory_order_release);
}

typedef struct {
    const a5o_table *t; const uint8_t *words; const uint64_t *off; size_t nw;
    int mode, mn, mx; chan_t ch; atomic_size_t next; atomic_int err; int fd;
    uint64_t out_cands, out_bytes;
    str_pool *pools;
} pipe_job;

typedef struct { pipe_job *j; int id; } pipe_worker_arg;

static void emit_chan(void *u, const uint8_t *s, size_t n) {
    pipe_worker_arg *w = (pipe_worker_arg *)u;
    chan_msg m;
    m.owner = n + 1 <= POOL_SLOT ? w->id : -1;
    if (m.owner >= 0) {
        m.v.p = pool_get(&w->j->pools[w->id]);
        if (n) memcpy(m.v.p, s, n);
        m.v.p[n] = 0; m.v.n = n;
    } else {
        m.v = bdup(s, n);
    }
    chan_send(&w->j->ch, m);   /* Go: newWord is a fresh string; out <- newWord */
}

static void *pipe_worker(void *arg) {
    pipe_worker_arg *w = (pipe_worker_arg *)arg;
    pipe_job *j = w->j;
    for (;;) {
        size_t i = atomic_fetch_add(&j->next, 1);
        if (i >= j->nw) break;
        int rc = a5o_expand_word(j->t, j->words + j->off[i], (size_t)(j->off[i + 1] - j->off[i]),
                                 j->mode, j->mn, j->mx, emit_chan, w);
        if (rc) atomic_store(&j->err, rc);
    }
    return NULL;
}

static void *pipe_writer(void *arg) {
    pipe_job *j = (pipe_job *)arg;
    uint8_t wb[4096]; size_t wn = 0; chan_msg m;
    while (chan_recv(&j->ch, &m)) {
        /* writer.WriteString(s + "\n"): the concat allocates a new string */
        bstr s = m.v;
        bstr line = bdup(s.p, s.n + 1); line.p[s.n] = '\n';
        if (m.owner >= 0) pool_put(&j->pools[m.owner], s.p);
        else free(s.p);
        size_t n = line.n, o = 0;
        while (o < n) {
            size_t k = sizeof(wb) - wn; if (k > n - o) k = n - o;
            memcpy(wb + wn, line.p + o, k); wn += k; o += k;
            if (wn == sizeof(wb)) { if (write(j->fd, wb, wn) < 0) {} wn = 0; }
        }
        j->out_cands++; j->out_bytes += n;
        free(line.p);
    }
    if (wn && write(j->fd, wb, wn) < 0) {}
    return NULL;
}

A5O_EXPORT int a5o_run_pipeline(const a5o_table *t, const uint8_t *words, const uint64_t *off, size_t nw,
                                int mode, int mn, int mx, int nthreads, int fd,
                                uint64_t *out_cands, uint64_t *out_bytes) {
    pipe_job *j = NULL;
    if (posix_memalign((void **)&j, 64, sizeof(pipe_job))) return -1;
    memset(j, 0, sizeof(pipe_job));
    j->t = t; j->words = words; j->off = off; j->nw = nw; j->mode = mode; j->mn = mn; j->mx = mx; j->fd = fd;
    chan_init(&j->ch);
    atomic_init(&j->next, 0); atomic_init(&j->err, 0);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t wr, th[256];
    pipe_worker_arg wa[256];
    j->pools = NULL;
    if (posix_memalign((void **)&j->pools, 64, (size_t)nthreads * sizeof(str_pool))) { free(j); return -1; }
    memset(j->pools, 0, (size_t)nthreads * sizeof(str_pool));
    for (int i = 0; i < nthreads; i++) {
        j->pools[i].ret = (uint8_t **)xrealloc(NULL, POOL_RET * sizeof(uint8_t *));
        atomic_init(&j->pools[i].rhead, 0); atomic_init(&j->pools[i].rtail, 0);
    }
    pthread_create(&wr, NULL, pipe_writer, j);
    for (int i = 0; i < nthreads; i++) { wa[i].j = j; wa[i].id = i; pthread_create(&th[i], NULL, pipe_worker, &wa[i]); }
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    chan_close(&j->ch);  /* close(out) after wg.Wait() */
    pthread_join(wr, NULL);
    *out_cands = j->out_cands; *out_bytes = j->out_bytes;
    int rc = atomic_load(&j->err);
    for (int i = 0; i < nthreads; i++) {
        for (size_t b = 0; b < j->pools[i].nblocks; b++) free(j->pools[i].blocks[b]);
        free(j->pools[i].blocks); free(j->pools[i].ret);
    }
    free(j->pools);
    free(j);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* Digest baseline: the reference expansion with   */
/* every candidate hashed where it is produced and probed in a target set --   */
/* the CPU shape of `a5_generator ... | hashcat -m 0/1000` without the pipe.   */
/* MD5 = RFC 1321 (Go crypto/md5); NTLM = RFC 1320 MD4 over Go's               */
/* utf16.Encode([]rune(s)) as UTF-16LE (invalid UTF-8 byte -> U+FFFD).         */
/* ------------------------------------------------------------------------ */
#define ROTL32(x, s) (((x) << (s)) | ((x) >> (32 - (s))))

static void md5_block(uint32_t h[4], const uint32_t M[16]) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
        0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
        0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
        0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
        0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
        0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
        0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
    static const int S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9, 14, 20, 5, 9, 14, 20, 5, 9, 14, 20, 5, 9, 14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f; int g;
        if (i < 16) { f = (b & c) | (~b & d); g = i; }
        else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
        else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
        else { f = c ^ (b | ~d); g = (7 * i) & 15; }
        uint32_t t = d; d = c; c = b;
        uint32_t x = a + f + K[i] + M[g];
        b = b + ROTL32(x, S[i]);
        a = t;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d;
}

static void md4_block(uint32_t h[4], const uint32_t X[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
#define F4(x, y, z) (((x) & (y)) | (~(x) & (z)))
#define G4(x, y, z) (((x) & (y)) | ((x) & (z)) | ((y) & (z)))
#define H4(x, y, z) ((x) ^ (y) ^ (z))
    static const int r2[16] = {0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15};
    static const int r3[16] = {0, 8, 4, 12, 2, 10, 6, 14, 1, 9, 5, 13, 3, 11, 7, 15};
    static const int s1[4] = {3, 7, 11, 19}, s2[4] = {3, 5, 9, 13}, s3[4] = {3, 9, 11, 15};
    for (int i = 0; i < 16; i++) {
        uint32_t t;
        switch (i & 3) {
        case 0: t = a + F4(b, c, d) + X[i]; a = ROTL32(t, s1[0]); break;
        case 1: t = d + F4(a, b, c) + X[i]; d = ROTL32(t, s1[1]); break;
        case 2: t = c + F4(d, a, b) + X[i]; c = ROTL32(t, s1[2]); break;
        default: t = b + F4(c, d, a) + X[i]; b = ROTL32(t, s1[3]); break;
        }
    }
    for (int i = 0; i < 16; i++) {
        uint32_t t, k = (uint32_t)r2[i];
        switch (i & 3) {
        case 0: t = a + G4(b, c, d) + X[k] + 0x5A827999u; a = ROTL32(t, s2[0]); break;
        case 1: t = d + G4(a, b, c) + X[k] + 0x5A827999u; d = ROTL32(t, s2[1]); break;
        case 2: t = c + G4(d, a, b) + X[k] + 0x5A827999u; c = ROTL32(t, s2[2]); break;
        default: t = b + G4(c, d, a) + X[k] + 0x5A827999u; b = ROTL32(t, s2[3]); break;
        }
    }
    for (int i = 0; i < 16; i++) {
        uint32_t t, k = (uint32_t)r3[i];
        switch (i & 3) {
        case 0: t = a + H4(b, c, d) + X[k] + 0x6ED9EBA1u; a = ROTL32(t, s3[0]); break;
        case 1: t = d + H4(a, b, c) + X[k] + 0x6ED9EBA1u; d = ROTL32(t, s3[1]); break;
        case 2: t = c + H4(d, a, b) + X[k] + 0x6ED9EBA1u; c = ROTL32(t, s3[2]); break;
        default: t = b + H4(c, d, a) + X[k] + 0x6ED9EBA1u; b = ROTL32(t, s3[3]); break;
        }
    }
#undef F4
#undef G4
#undef H4
    h[0] += a; h[1] += b; h[2] += c; h[3] += d;
}

/* Merkle-Damgard over msg (little-endian words, 0x80 pad, 64-bit bit length): MD5 or MD4 */
static __attribute__((noinline)) void md_message(int md5, const uint8_t *msg, size_t n, uint8_t out[16]) {
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    uint32_t M[16];
    const size_t full = n / 64;
    for (size_t b = 0; b < full; b++) {
        memcpy(M, msg + 64 * b, 64);
        if (md5) md5_block(h, M); else md4_block(h, M);
    }
    uint8_t tail[128];
    memset(tail, 0, sizeof tail);
    const size_t r = n - 64 * full;
    memcpy(tail, msg + 64 * full, r);
    tail[r] = 0x80;
    const size_t tb = r < 56 ? 64 : 128;
    const uint64_t bits = (uint64_t)n * 8;
    memcpy(tail + tb - 8, &bits, 8);
    for (size_t o = 0; o < tb; o += 64) {
        memcpy(M, tail + o, 64);
        if (md5) md5_block(h, M); else md4_block(h, M);
    }
    memcpy(out, h, 16);
}

/* Go utf16.Encode([]rune(s)) as UTF-16LE bytes; returns the byte count (out >= 4 n) */
static size_t go_utf16le(const uint8_t *s, size_t n, uint8_t *out) {
    size_t i = 0, o = 0;
    while (i < n) {
        int sz, r = decode_rune(s + i, n - i, &sz);
        i += (size_t)sz;
        if (r >= 0x10000) {
            uint32_t v = (uint32_t)r - 0x10000u, hi = 0xD800u + (v >> 10), lo = 0xDC00u + (v & 0x3FFu);
            out[o++] = (uint8_t)hi; out[o++] = (uint8_t)(hi >> 8); out[o++] = (uint8_t)lo; out[o++] = (uint8_t)(lo >> 8);
        } else {
            out[o++] = (uint8_t)r; out[o++] = (uint8_t)((unsigned)r >> 8);
        }
    }
    return o;
}

/* algo 0: MD5(s); 1: NTLM(s) = MD4(UTF-16LE(s)) */
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wmaybe-uninitialized"  /* (stackbuf: written by go_utf16le first) */
A5O_EXPORT int a5o_digest(int algo, const uint8_t *s, size_t n, uint8_t out[16]) {
    if (algo == 0) { md_message(1, s, n, out); return A5O_OK; }
    if (algo != 1) return A5O_E_ARG;
    uint8_t stackbuf[1024];
    uint8_t *u = 4 * n <= sizeof stackbuf ? stackbuf : (uint8_t *)malloc(4 * n + 1);
    if (!u) return A5O_E_NOMEM;
    size_t m = go_utf16le(s, n, u);
    md_message(0, u, m, out);
    if (u != stackbuf) free(u);
    return A5O_OK;
}
#pragma GCC diagnostic pop

/* target set: open addressing on the first 8 digest bytes */
typedef struct {
    const a5o_table *t; const uint8_t *words; const uint64_t *off; size_t nw;
    int mode, mn, mx, algo;
    const uint8_t *tg; const int64_t *slot; size_t smask;
    _Atomic size_t next; _Atomic int err;
    _Atomic uint64_t cands, hits;
} dg_job;
typedef struct { dg_job *j; uint64_t cands, hits; } dg_local;

static void emit_hash_probe(void *u, const uint8_t *s, size_t n) {
    dg_local *L = (dg_local *)u;
    uint8_t d[16];
    a5o_digest(L->j->algo, s, n, d);
    uint64_t k; memcpy(&k, d, 8);
    for (size_t i = fmix64(k) & L->j->smask;; i = (i + 1) & L->j->smask) {
        int64_t x = L->j->slot[i];
        if (x < 0) break;
        if (!memcmp(L->j->tg + 16 * (size_t)x, d, 16)) { L->hits++; break; }
    }
    L->cands++;
}

static void *dg_worker(void *arg) {
    dg_job *j = (dg_job *)arg;
    dg_local L = {j, 0, 0};
    for (;;) {
        size_t i = atomic_fetch_add(&j->next, 16);
        if (i >= j->nw) break;
        size_t e = i + 16 < j->nw ? i + 16 : j->nw;
        for (; i < e; i++) {
            int rc = a5o_expand_word(j->t, j->words + j->off[i], (size_t)(j->off[i + 1] - j->off[i]), j->mode, j->mn,
                                     j->mx, emit_hash_probe, &L);
            if (rc) atomic_store(&j->err, rc);
        }
    }
    atomic_fetch_add(&j->cands, L.cands);
    atomic_fetch_add(&j->hits, L.hits);
    return NULL;
}

/* nthreads workers (one word at a time, like the reference's goroutines), each candidate
 * digested and probed in a hash set of the nt 16-B targets; returns candidates and hits */
A5O_EXPORT int a5o_digest_run(const a5o_table *t, const uint8_t *words, const uint64_t *off, size_t nw, int mode,
                              int mn, int mx, int algo, const uint8_t *targets, size_t nt, int nthreads,
                              uint64_t *out_cands, uint64_t *out_hits) {
    if (algo != 0 && algo != 1) return A5O_E_ARG;
    size_t ns = 16;
    while (ns < 2 * nt + 16) ns <<= 1;
    int64_t *slot = (int64_t *)malloc(ns * sizeof(int64_t));
    if (!slot) return A5O_E_NOMEM;
    for (size_t i = 0; i < ns; i++) slot[i] = -1;
    for (size_t x = 0; x < nt; x++) {
        uint64_t k; memcpy(&k, targets + 16 * x, 8);
        size_t i = fmix64(k) & (ns - 1);
        while (slot[i] >= 0) i = (i + 1) & (ns - 1);
        slot[i] = (int64_t)x;
    }
    dg_job j;
    j.t = t; j.words = words; j.off = off; j.nw = nw; j.mode = mode; j.mn = mn; j.mx = mx; j.algo = algo;
    j.tg = targets; j.slot = slot; j.smask = ns - 1;
    atomic_init(&j.next, 0); atomic_init(&j.err, 0); atomic_init(&j.cands, 0); atomic_init(&j.hits, 0);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, dg_worker, &j);
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    free(slot);
    *out_cands = atomic_load(&j.cands);
    *out_hits = atomic_load(&j.hits);
    return atomic_load(&j.err);
}
