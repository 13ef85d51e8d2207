// mb_rounds.hip -- rounds-only throughput of the k_expand_fast round machinery
// (fx_rounds / fx_round / fb_put / fx_flush of a5x_kernels.hip) on a synthetic
// resident window: no window setup, no metadata, no records.  Tells how much of the
// kernel's time the rounds alone would take at the C3 shape.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I hashcat_a5_table_generator_amd/csrc \
//        tools/mb_rounds.hip -o tools/mb_rounds
#include "../hashcat_a5_table_generator_amd/csrc/a5x_kernels.hip"
#include "../hashcat_a5_table_generator_amd/csrc/a5x_fx6.h"

#include <stdio.h>
#include <stdlib.h>
#include <string>
#include <string.h>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

struct MbArgs {
  uint8_t* out;
  u64 region;   // bytes per wave
  u32 nwords;   // window words
  u32 R[4];     // big piece R (1 past NB)
  u32* err;
  u64* dbg;
  u64* written;
  int nostore;
};

// ---- v6 rounds ----
struct Mb6Flush {
  uint8_t* out;
  u32* ring;
  bool nostore;
  __device__ __forceinline__ void operator()(FxRun& R) {
    const u32 lane = lane_id();
    const u32 nb = uniform((u32)((R.pos - R.B) >> 4));
    if (nb == 0) return;
    const u64 B = uniform64(R.B);
    const uint4* r4 = (const uint4*)ring;
    if (!nostore)
      for (u32 b = lane; b < nb; b += 64) *(uint4*)(out + B + 16ull * b) = r4[b];
    if (lane == 0) ((uint4*)ring)[0] = r4[nb];
    R.B = B + 16ull * nb;
    WAVE_SYNC();
  }
};

template <int K> constexpr u32 ring6() { return K == 4 ? 4224u : (K == 3 ? 3200u : 2176u); }
template <int K> constexpr u32 lds6_per_wave() { return (ring6<K>() + 256 + (u32)sizeof(FXWin) + 15u) & ~15u; }

template <int NB, int WPE, int K>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) k_mb6(MbArgs m) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const u32 wv = uniform(threadIdx.x / 64), lane = lane_id();
  uint8_t* mine = smem + wv * lds6_per_wave<K>();
  u32* ring = (u32*)mine;
  FXWin& F = *(FXWin*)(mine + ring6<K>() + 256);
  u32 E = 0, P = 1;
  for (int b = 0; b < 4; b++) { E += b < NB ? m.R[b] : 0; P *= b < NB ? m.R[b] : 1; }
  const u32 cnt = P - 1;
  const u32 k = m.nwords;
  for (u32 t = lane; t < k * E; t += 64) {
    const u32 j = t / E;
    u32 u = t - j * E, b = 0;
    while (u >= m.R[b]) { u -= m.R[b]; b++; }
    u32 len = 4 + (u + j) % 5;
    u32 w[4] = {0, 0, 0, 0};
    for (u32 i = 0; i < len; i++) {
      u32 ch = (b == NB - 1 && i == len - 1) ? 10u : (u32)('a' + (i + u + b) % 26);
      w[i >> 2] |= ch << (8 * (i & 3));
    }
    w[3] |= len << 24;
    F.be[t] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  if (lane == 0) F.be[FX6_ZBE] = make_uint4(0, 0, 0, 0);
  const u32 maxl = NB * 8;
  const u32 runs_w = (cnt + K - 1) / K;
  if (lane < k) {
    const u32 eb = lane * E;
    u32 rm = 0, eb4[4] = {FX6_ZBE, FX6_ZBE, FX6_ZBE, FX6_ZBE}, mg[4] = {0, 0, 0, 0}, acc = eb;
    for (int b = 0; b < NB; b++) { rm |= (m.R[b] - 1u) << (6 * b); eb4[b] = acc; acc += m.R[b]; mg[b] = fr_magic(m.R[b]); }
    F.wq[lane][0] = make_uint4(mg[0], mg[1], mg[2], mg[3]);
    F.wq[lane][1] = make_uint4(rm, eb4[0] | (eb4[1] << 16), eb4[2] | (eb4[3] << 16), lane * runs_w);
    F.rb[lane] = 0;
    F.re[lane] = cnt;
  }
  WAVE_SYNC();
  const u64 wid = (u64)blockIdx.x * (blockDim.x / 64) + wv;
  const u64 base = wid * m.region;
  FxRun R;
  R.B = base; R.lo = base; R.pos = base; R.carry = 0; R.open = true;
  Mb6Flush fl;
  fl.out = m.out;
  fl.ring = ring;
  fl.nostore = m.nostore;
  const u32 truns = k * runs_w;
  const u32 rw = lane < k ? lane * runs_w : 0xffffffffu;
  const u32 ringa = fx6_addr(ring), trash = ringa + ring6<K>() + 4u * lane;
  const u64 winbytes_max = (u64)k * cnt * maxl;
  while (R.pos + winbytes_max + 64 < base + m.region) {
    u32 jcur = 0;
    for (u32 rr = 0; rr < truns; rr += 64) {
      const u32 j = fx6_word(rw, k, rr, 64u, jcur);
      const u32 took = fx6_round<NB, K>(F.be, F.wq, F.rb, F.re, ringa, trash, ring6<K>() - 32u, R, rr, j,
                                        rr + lane < truns, fl);
      rr += took - 64u;
    }
  }
  // close: flush the partial tail block (microbench: whole block)
  if (R.pos & 3u) { if (lane == 0) ring[(u32)(R.pos - R.B) >> 2] = R.carry; }
  WAVE_SYNC();
  if (lane == 0 && R.pos > R.B) *(uint4*)(m.out + R.B) = ((const uint4*)ring)[0];
  if (lane == 0) atomicAdd((unsigned long long*)m.written, (unsigned long long)(R.pos - base));
}

template <int NB, int WPE, int K>
void run6(const char* name, MbArgs m, u32 nwaves) {
  constexpr u32 wpb = 4;
  const size_t lds = wpb * lds6_per_wave<K>();
  CHK(hipFuncSetAttribute((const void*)k_mb6<NB, WPE, K>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  float best = 1e30f;
  u64 wr = 0;
  for (int it = 0; it < 4; it++) {
    CHK(hipMemset(m.written, 0, 8));
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_mb6<NB, WPE, K>), dim3(nwaves / wpb), dim3(64 * wpb), lds, 0, m);
    CHK(hipGetLastError());
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
    CHK(hipMemcpy(&wr, m.written, 8, hipMemcpyDeviceToHost));
  }
  printf("v6 %-11s K=%d NB=%d wpe=%d lds/wave=%u R={%u,%u,%u,%u}: %.3f GB in %.3f ms = %.0f GB/s\n", name, K, NB, WPE,
         lds6_per_wave<K>(), m.R[0], m.R[1], m.R[2], m.R[3], wr / 1e9, best, wr / (best * 1e-3) / 1e9);
}

// verification: the v6 output of wave 0 vs a host re-enumeration of the synthetic window
int verify6(MbArgs m) {
  const u32 NB = 2;
  u32 E = m.R[0] + m.R[1], P = m.R[0] * m.R[1], cnt = P - 1;
  std::vector<std::string> ent(m.nwords * E);
  for (u32 t = 0; t < m.nwords * E; t++) {
    const u32 j = t / E;
    u32 u = t - j * E, b = 0;
    while (u >= m.R[b]) { u -= m.R[b]; b++; }
    u32 len = 4 + (u + j) % 5;
    std::string x;
    for (u32 i = 0; i < len; i++) x += (char)((b == NB - 1 && i == len - 1) ? 10 : ('a' + (i + u + b) % 26));
    ent[t] = x;
  }
  std::string win;
  for (u32 j = 0; j < m.nwords; j++)
    for (u32 n = 1; n <= cnt; n++) win += ent[j * E + n % m.R[0]] + ent[j * E + m.R[0] + n / m.R[0]];
  std::vector<char> h(m.region);
  CHK(hipMemcpy(h.data(), m.out, m.region, hipMemcpyDeviceToHost));
  u64 bad = 0, nwin = 0;
  for (u64 off = 0; off + win.size() <= m.region / 2; off += win.size(), nwin++)
    if (memcmp(h.data() + off, win.data(), win.size())) { bad++; if (bad < 3) {
      for (u64 i = 0; i < win.size(); i++) if (h[off + i] != win[i]) { printf("  first diff window %llu byte %llu: got %02x want %02x\n", (unsigned long long)nwin, (unsigned long long)i, (uint8_t)h[off+i], (uint8_t)win[i]); break; } } }
  printf("v6 verify: %llu of %llu windows differ\n", (unsigned long long)bad, (unsigned long long)nwin);
  return bad != 0;
}

static size_t lds_per_wave_fast_host() { return (FX_RING + FX_TRASH + sizeof(FXWin) + 15u) & ~(size_t)15u; }

// write roofline: every wave streams its region with 16-B stores (1 KiB per instruction)
__global__ void __launch_bounds__(256) k_store(uint8_t* out, u64 region) {
  const u64 wid = (u64)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  uint4* p = (uint4*)(out + wid * region);
  const uint4 v = make_uint4(threadIdx.x, 1, 2, 3);
  for (u64 i = lane_id(); i < region / 16; i += 64) p[i] = v;
}

int main(int argc, char** argv) {
  const u64 total = (u64)16 << 30;
  const u32 nwaves = 16384;
  MbArgs m;
  CHK(hipMalloc(&m.out, total + 4096));
  CHK(hipMalloc(&m.err, 256));
  CHK(hipMemset(m.err, 0, 256));
  m.dbg = (u64*)(m.err + 16);
  CHK(hipMalloc(&m.written, 8));
  m.region = total / nwaves;
  m.nwords = 8;
  m.R[0] = 13; m.R[1] = 14; m.R[2] = 1; m.R[3] = 1;
  m.nwords = 12;
  m.nwords = 9;
  m.nostore = 0;
  run6<2, 4, 4>("c3-like", m, nwaves);
  int vbad = verify6(m);
  run6<2, 4, 3>("c3-like", m, nwaves);
  vbad |= verify6(m);
  run6<2, 4, 2>("c3-like", m, nwaves);
  vbad |= verify6(m);
  run6<2, 2, 4>("c3-like", m, nwaves);
  run6<2, 1, 4>("c3-like wpe1", m, nwaves);
  {
    MbArgs m3 = m;
    m3.R[0] = 6; m3.R[1] = 6; m3.R[2] = 5; m3.R[3] = 1; m3.nwords = 14;
    run6<3, 2, 4>("3 pieces", m3, nwaves);
    m3.R[0] = 4; m3.R[1] = 4; m3.R[2] = 4; m3.R[3] = 3; m3.nwords = 16;
    run6<4, 2, 4>("4 pieces", m3, nwaves);
  }
  m.nostore = 1;
  run6<2, 2, 4>("nostore", m, nwaves);
  m.nostore = 0;
  {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int it = 0; it < 4; it++) {
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_store, dim3(nwaves / 4), dim3(256), 0, 0, m.out, m.region);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms = 0;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    printf("store roofline: %.3f GB in %.3f ms = %.0f GB/s\n", total / 1e9, best, total / (best * 1e-3) / 1e9);
  }
  return vbad;
}
