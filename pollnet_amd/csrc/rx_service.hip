// Resident classify service (round 5): one launch, then the host posts batches through pinned host
// memory and the kernel -- already on the GPU -- classifies each with the production code (classify_group,
// rx_classify.hpp), without a launch per batch.  A launch costs ≈7 µs of host-to-GPU round trip; a resident wave
// answering a doorbell ≈2.7 µs (bench/bench_doorbell, profiles/r05/latency/).
//
// Protocol (round 6: every wave reads the mailbox itself).  Two mailbox slots of one 64-B line each, then a line
// holding the exit flag; post k uses slot k & 1.  On a large-BAR device (MI355X) the mailbox is uncached device
// memory that the host writes through the BAR, so a post lands in HBM and every wave of the kernel, on every XCD, sees
// it with its own read of device memory -- no wave hands a post to the others.  (Without a large BAR the mailbox is
// pinned host memory and the waves other than 0 poll it less often.)  The host writes a slot's fields and their check
// word, store fence, then its first word (gen) and last word (seq) = k, store fence.  Each wave keeps the last post it
// saw and reads both slots and the exit flag with one load (lanes 0-31: the slots, lane 32: the flag); it waits for the
// next post, last + 1, in that post's slot, whole (gen = seq = k, the check word matching, so a read that mixed two
// posts' words is refused) -- never taking a later post from the other slot first, since its read of the next post's
// slot may be the older one.  A slot holding a later post means the next post was complete without this wave: the wave
// was not one of its waves and passes it.  A post runs on its first `act` waves (one per group of frames, at most all of
// them; svc_fpw sizes the groups); the others note it went by.  A wave takes posts in order, so it never skips a post
// it runs on: the host reuses post k's slot (for post k + 2) only once post k is complete (a wave that took post k + 1
// from the other slot before post k would store done word k + 1 without having run post k).  Each wave of a post makes
// its records system-visible and stores k to its own host done word; the host waits on the words of the post's waves.
// A post completing through done word 0 alone -- a linked post (its chain pass runs after every wave's records) or a
// large one (on more waves than there are done words) -- is counted on a per-slot device counter, and its last wave
// completes it.  Posts k and k + 1 may run at once on different waves.  A stop post (n = PN_SERVICE_STOP) ends every
// wave.  After idle_ms without a post wave 0 stores the launch's epoch to the exit flag and to the host's exit word and
// ends; the others end on the flag (a safety limit of their own backs it); the host relaunches on its next post, and a
// post the ended launch left incomplete runs again.  So the kernel always ends.
// Large posts (round 6).  The resident kernel is the latency tier: kLatWaves (64) one-wave workgroups, which answer
// every post of up to 4096 frames and leave the rest of the chip to other kernels while idle.  A post above that
// also runs on helper waves: a grid the host launches with the post on a stream of its own (a launch's ~7 us is
// nothing beside a large post's run).  The helpers get the post in their arguments, take their share of its groups as
// waves kLatWaves.. of it and end -- no wait, no count, no write-back of their own: the host takes the post as done
// once the resident waves' done word and the helper grid's end are both there.  The slot's fpw word carries the
// helper count (bits 8+), so the resident waves know the post's wave count.  Only vector memory operations
// (global loads / stores / one atomic add).
#include <algorithm>
#include <chrono>
#include <cstdlib>

#include "rx_classify.hpp"

namespace {
using pn_internal::hip_err;
using pn_internal::set_err;

struct alignas(64) SvcPost { // one 64-B line: a mailbox slot (host) or its device copy
  uint32_t gen;              // = seq, stored after the fields
  uint32_t n;                // frames | kPostVerify | kPostLinks, or PN_SERVICE_STOP
  uint32_t fpw;              // frames per group (svc_fpw, bits 0-7) | helper waves << 8 (svc_helpers)
  uint32_t max_conn;
  const uint8_t* frames;
  pn_result* out;
  const pn_conn_entry* tbl;
  uint16_t* links;           // pn_service_post_linked: the chain links (host or device memory), else nullptr
  uint32_t mask;             // tbl_mask (< n_entries: 32 bits)
  uint32_t n_entries;
  uint32_t check; // svc_check: k ^ the xor of words 1-13, so a read that mixed two posts' words is refused
  uint32_t seq; // stored last (release)
};
static_assert(sizeof(SvcPost) == 64, "one line per post");

constexpr uint32_t kDoneWords = 64; // host words: one done word per wave of a post on at most this many waves,
constexpr uint32_t kCountWords = 64; // then one per mailbox slot for counted posts (completed by their last wave),
constexpr uint32_t kExitWord = 96;   // then the exit word on a line of its own
constexpr uint32_t kWordsBytes = 512;
constexpr uint32_t kLatWaves = PN_SERVICE_WAVES; // the latency tier: every post of up to 4096 frames runs on these
static_assert(kLatWaves <= kDoneWords, "a latency-tier post completes through per-wave done words");
constexpr uint32_t kLatFrames = kLatWaves * kFramesPerWave; // the largest post the tier takes alone
constexpr uint32_t kNetLimitMs = 8000; // waves other than 0: ended after 1.5 x idle_ms + this without a post, should
                                       // wave 0's exit flag never come (pn_service_wait gives up at 10 s)
constexpr uint32_t kPostVerify = 1u << 30, kPostLinks = 1u << 29, kPostN = (1u << 21) - 1; // the n word
constexpr uint32_t kLinkFrames = PN_LINK_MAX_FRAMES, kLinkConns = PN_LINK_MAX_CONNS;
constexpr uint32_t kMailBytes = 4096; // the mailbox allocation: slot 0, slot 1, the exit flag's line
// Post ids count up by one and wrap (2^32 posts: 11 hours at 100k posts/s): every 32-bit value is a post's id, and
// "after" is the wrap-aware order.  A stop post is marked by its n word.

struct alignas(64) SvcDev { // device memory, set by the host before every launch
  uint32_t count[2][16];    // per mailbox slot (one line each): the resident waves done with its post (counted posts)
};
constexpr uint32_t kExitFlag = 32; // the mailbox's word 32 (its third line): the epoch of the launch whose wave 0 ended

// Measurement build only (-DPN_SVC_TRACE, bench/svc_trace.cpp): lane 0 of each wave stores the device wall clock at
// the protocol's steps to pinned host memory (pn_svc_trace_set); compiled out of the product.  Plain stores: a step
// before the wave's system fence reaches the host with the post, a later one only with the next post's fence.
#ifdef PN_SVC_TRACE
__device__ uint64_t* g_svc_trace = nullptr;
#define SVC_T(w, i)                                                       \
  do {                                                                    \
    if (lane == 0 && (w) < 64) g_svc_trace[(w) * 8 + (i)] = wall_clock64(); \
  } while (0)
#else
#define SVC_T(w, i) \
  do {              \
  } while (0)
#endif

struct SArgs {
  const SvcPost* mail;  // the two mailbox slots, then the exit flag's line (device memory, or pinned host)
  u32x4* scratch;       // device: per mailbox slot, kLinkFrames x 2 chain entries (kChainAux)
  uint32_t* done_words; // host: per wave, the last post it finished its groups of
  uint32_t* exit_word;  // host: the launch's epoch once it ended for lack of posts
  SvcDev* dev;
  uint64_t idle_ticks; // device wall clock
  uint64_t net_ticks;  // waves other than 0: their own limit without a post, should wave 0's flag never come
  uint32_t epoch;
  uint32_t last; // the post completed before this launch
  uint32_t stride, ipa_off, avail;
  uint32_t poll_sleep; // waves other than 0: s_sleep between reads of the mailbox (1 in device memory)
};

// Frames per group (host, at the post).  The release path reads one header line per frame: 64 frames a wave, so a
// post of up to 64 frames is wave 0's alone (no cross-wave step at all).  Verifying reads every byte: a small
// post is spread over more waves of the latency tier (8 frames a group and up, as few waves' worth of streaming as
// the post allows).  A post above the tier's 64 groups of 64 frames runs 64-frame groups on every wave.
inline uint32_t svc_fpw(uint32_t n, bool verify) {
  uint32_t fpw = verify ? 8u : kFramesPerWave;
  while (fpw < kFramesPerWave && (n + fpw - 1) / fpw > kLatWaves) fpw <<= 1;
  return fpw;
}

// The slot's check word for post k over its words 1-13 (n .. fpw).
inline uint32_t svc_check(const SvcPost* p, uint32_t k) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
  uint32_t x = k;
  for (int i = 1; i <= 13; i++) x ^= w[i];
  return x;
}

// the waves a post runs on: one per group, at most all (the host computes the same)
__host__ __device__ __forceinline__ uint32_t svc_active(uint32_t n, uint32_t fpw, uint32_t waves) {
  const uint32_t groups = (n + fpw - 1) / fpw;
  return groups < waves ? groups : waves;
}

// helper waves of a post (host): none up to kLatFrames, else one per group past the tier's, at most `max`
inline uint32_t svc_helpers(uint32_t n, uint32_t max) {
  if (n <= kLatFrames) return 0;
  const uint32_t groups = (n + kFramesPerWave - 1) / kFramesPerWave;
  return std::min(groups - kLatWaves, max);
}

// a post's kernel arguments from its 64-B line held one word per lane (lanes b .. b + 15, SvcPost's layout)
__device__ __forceinline__ KArgsAux svc_args(uint32_t v, uint32_t b, const SArgs& s, uint32_t k) {
  // readlane returns int: each word through uint32_t, or a low word with bit 31 set would sign-extend
  auto w32 = [&](uint32_t i) { return (uint32_t)__builtin_amdgcn_readlane(v, b + i); };
  auto u64 = [&](uint32_t lo) { return ((uint64_t)w32(lo + 1) << 32) | w32(lo); };
  KArgsAux a;
  const uint32_t nw = w32(1);
  a.n = nw & kPostN;
  a.fpw = w32(2) & 0xffu;
  a.max_conn = w32(3);
  a.frames = reinterpret_cast<const uint8_t*>(u64(4));
  a.out = reinterpret_cast<pn_result*>(u64(6));
  a.tbl = reinterpret_cast<const pn_conn_entry*>(u64(8));
  a.mask = w32(12);
  a.n_entries = w32(13);
  a.stride = s.stride;
  a.ipa_off = s.ipa_off;
  a.avail = s.avail;
  a.offs = nullptr;
  // a linked post's frames also leave their chain entries in the slot's scratch
  a.aux = (nw & kPostLinks) ? s.scratch + (size_t)(k & 1) * kLinkFrames * 2 : nullptr;
  return a;
}

__device__ __forceinline__ uint16_t* svc_links(uint32_t v, uint32_t b) {
  return reinterpret_cast<uint16_t*>(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(v, b + 11) << 32) |
                                     (uint32_t)__builtin_amdgcn_readlane(v, b + 10));
}

// ---- chain links (round 6): the in-order successor structure of a post, for the host's fast path ----
// links[i] = d > 0 when frame j = i - d is the previous frame of the same connection in the post (records with
// PN_F_HIT and not PN_F_TW; other frames are not part of any chain) and frame i continues it exactly: both frames
// are clean (ACK; no SYN, FIN, RST; no NOT_TCP / TRUNC / BADOFF / IHL_NE_5; IP_OK and TCP_OK or TCP_UNCHECKED),
// both carry payload, seq_i = seq_j + payload_len_j, and payload offset, ack number, window, destination address and
// port are equal.  Else 0.  The oracle's statement is orc_chain_links (oracle/pn_oracle.c).
constexpr uint32_t kCleanNeed = PN_F_HIT | PN_F_ACK | PN_F_IP_OK;
constexpr uint32_t kCleanNone = PN_F_TW | PN_F_SYN | PN_F_FIN | PN_F_RST | PN_F_NOT_TCP | PN_F_TRUNC | PN_F_BADOFF |
                                PN_F_IHL_NE_5;

struct ChainLds {
  uint32_t last[kLinkConns]; // 1 + the last frame of each connection so far (0: none)
  uint32_t key[kLinkFrames]; // each frame's connection (0xFFFFFFFF: in no chain), to reset `last` after the pass
  uint32_t seq_end[kLinkFrames];
  u32x4 fields[kLinkFrames]; // ack, dst_ip, window | dst_port, payload_off | usable << 16
};

__device__ __forceinline__ ChainLds& chain_lds() {
  __shared__ ChainLds c;
  return c;
}

// every entry of the table: none (at launch; each pass resets what it used)
__device__ __forceinline__ void chain_init(int lane) {
  ChainLds& c = chain_lds();
  for (uint32_t i = lane; i < kLinkConns; i += kWave) c.last[i] = 0u;
  wave_lds_sync();
}

// One 64-frame step of the pass: frame i = base + lane with its record and chain fields (rec, fx; i < n when valid).
__device__ __forceinline__ void chain_step(ChainLds& c, uint32_t base, uint32_t n, uint32_t max_conn, bool on,
                                           const u32x4& rec, const u32x4& fx, const __amdgpu_buffer_rsrc_t& lr,
                                           uint64_t below, int lane) {
  const uint32_t i = base + lane;
  const bool valid = i < n;
  const uint32_t flags = rec.w & 0xffffu;
  const uint32_t len = rec.z >> 16; // payload_len (int16): usable when in (0, 0x8000)
  const bool member = on && valid && (flags & (PN_F_HIT | PN_F_TW)) == PN_F_HIT && rec.x < max_conn;
  const bool usable = (flags & kCleanNeed) == kCleanNeed && (flags & kCleanNone) == 0 &&
                      (flags & (PN_F_TCP_OK | PN_F_TCP_UNCHECKED)) != 0 && len != 0 && len < 0x8000u;
  const uint32_t key = member ? rec.x : 0u;
  if (valid) { // this frame's fields, for its successor
    c.key[i] = member ? key : 0xFFFFFFFFu;
    c.seq_end[i] = rec.y + len;
    c.fields[i] = u32x4{fx.x, fx.y, fx.z, (rec.z & 0xffffu) | (usable ? 0x10000u : 0u)};
  }
  uint32_t prev = 0; // 1 + the previous frame, 0 = none
  if (member) prev = c.last[key];
  wave_lds_sync();
  if (member) atomicMax(&c.last[key], i + 1);
  wave_lds_sync();
  uint64_t todo = __ballot(member && c.last[key] != i + 1); // lanes with a higher lane of their connection
  while (todo) {
    const uint32_t leader = (uint32_t)__builtin_ctzll(todo);
    const uint32_t kk = __builtin_amdgcn_readlane(key, leader);
    const uint64_t m = __ballot(member && key == kk);
    todo &= ~m;
    const uint64_t lower = m & below;
    if (member && key == kk && lower) prev = base + 64u - (uint32_t)__builtin_clzll(lower); // 1 + that lane
  }
  uint32_t d = 0;
  if (member && usable && prev) {
    const uint32_t j = prev - 1;
    const u32x4 pf = c.fields[j];
    if ((pf.w >> 16) && c.seq_end[j] == rec.y && pf.x == fx.x && pf.y == fx.y && pf.z == fx.z &&
        (pf.w & 0xffffu) == (rec.z & 0xffffu))
      d = i - j;
  }
  if (valid) __builtin_amdgcn_raw_buffer_store_b16((unsigned short)d, lr, i * 2, 0, 0);
  wave_lds_sync(); // this step's reads of fields before the next step's writes (other lanes' entries)
}

// The pass over a post's n frames (their chain entries in scratch `aux`, written by the post's waves and visible to
// this one), by one wave, in 64-frame steps: each frame's previous frame of its connection comes from the table of
// last frames -- or, where a connection repeats inside the step, from the highest lane below with the same
// connection (one ballot round per repeating connection: none in a step of distinct flows, one for a single flow).
// The entries are loaded 8 steps (512 frames) at a time, all in flight before the first is used: one memory round
// trip per 512 frames, not one per step.
__device__ __forceinline__ void chain_pass(const u32x4* aux, uint32_t n, uint32_t max_conn, uint16_t* links, int lane) {
  constexpr int kChunk = 8;
  ChainLds& c = chain_lds();
  const bool on = max_conn <= kLinkConns;
  const __amdgpu_buffer_rsrc_t lr = frame_rsrc(reinterpret_cast<const uint8_t*>(links), n * 2);
  const __amdgpu_buffer_rsrc_t ar = frame_rsrc(reinterpret_cast<const uint8_t*>(aux), n * 32);
  const uint64_t below = (1ull << lane) - 1;
  for (uint32_t base0 = 0; base0 < n; base0 += kChunk * kWave) {
    u32x4 rec[kChunk], fx[kChunk];
#pragma unroll
    for (int s = 0; s < kChunk; ++s) { // past n: the descriptor's range returns zeros (a miss: in no chain)
      const uint32_t i = base0 + s * kWave + lane;
      rec[s] = __builtin_amdgcn_raw_buffer_load_b128(ar, i * 32, 0, 0);
      fx[s] = __builtin_amdgcn_raw_buffer_load_b128(ar, i * 32 + 16, 0, 0);
    }
#pragma unroll
    for (int s = 0; s < kChunk; ++s)
      if (base0 + s * kWave < n) chain_step(c, base0 + s * kWave, n, max_conn, on, rec[s], fx[s], lr, below, lane);
  }
  // the table back to none for the next post (only the connections this one touched)
  for (uint32_t i = lane; i < n; i += kWave) {
    const uint32_t k = c.key[i];
    if (k != 0xFFFFFFFFu) c.last[k] = 0u;
  }
  wave_lds_sync();
}

// wave w's groups of the post (round robin over the post's waves), then its records made visible to the host and,
// on a post of at most kDoneWords waves without links, post k stored to its done word (a linked post completes after
// its chain pass, svc_finish)
// A helper wave (HELPER) makes nothing visible itself: its grid's end does (the host waits for it, svc_post_done),
// which spares the post one L2 write-back per helper wave.
template <int MIS, int COOP, bool HELPER = false>
__device__ __forceinline__ void svc_run(const KArgsAux& a, bool verify, bool linked, uint32_t w, uint32_t act, uint32_t k,
                                        uint32_t* done_word, int lane) {
  for (uint32_t g = w; g * a.fpw < a.n; g += act) {
    if (verify) classify_group<MIS, COOP, kProdAbl | kChainAux, kLoadAux, kStoreAux, 0, kLoadAux>(a, g * a.fpw, lane, nullptr);
    else
      classify_group<MIS, COOP, kProdAbl | kHeaderOnly | kChainAux, kLoadAux, kStoreAux, 0, kLoadAux>(a, g * a.fpw, lane,
                                                                                                     nullptr);
  }
  if constexpr (HELPER) return;
  __threadfence_system();
  if (lane == 0 && act <= kDoneWords && !linked)
    __hip_atomic_store(done_word, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The wave that completes a counted post (on more than kDoneWords waves, or linked) through its slot's count word
// (host words kCountWords + slot, never a wave's own done word: a wave may already run the next post): a linked post's
// chain pass first, over the chain entries every wave of the post left in scratch; then k to the count word once
// everything the post writes is visible to the host.
template <bool PASS>
__device__ __forceinline__ void svc_finish(const KArgsAux& a, uint16_t* links, uint32_t k, uint32_t* count_word, int lane) {
  if constexpr (PASS) {
    if (a.aux) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); // the other waves' chain entries
      chain_pass(a.aux, a.n, a.max_conn, links, lane);
    }
  }
  __threadfence_system();
  if (lane == 0) __hip_atomic_store(count_word, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// a counted post (linked, or on more than kDoneWords waves): count this wave done on its slot's counter; the last of
// the post's resident waves resets the counter (the slot's next post, k + 2, is issued only once k is complete) and
// completes the post through done word 0 (svc_finish).  Every wave's records and chain entries were made
// system-visible before its count, which pairs them with what the last wave does next.  A large post's helpers run
// beside the resident waves and do not count.
template <bool PASS>
__device__ __forceinline__ void svc_count(uint32_t* count, const KArgsAux& a, uint16_t* links, uint32_t target, uint32_t k,
                                          uint32_t* count_word, int lane) {
  uint32_t prev = 0;
  if (lane == 0) prev = atomicAdd(count, 1u);
  prev = __builtin_amdgcn_readfirstlane(prev);
  if (prev == target - 1) {
    if (lane == 0) __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); // before done word 0
    svc_finish<PASS>(a, links, k, count_word, lane);
  }
}

// Every wave reads the mailbox itself (one load: lanes 0-31 the two slots, lane 32 the exit flag) and takes the posts
// after the last one it saw, in order; it runs its groups of the posts it is one of the first `act` waves of.  Wave 0
// ends after idle_ms without a post (the idle limit runs from the end of its last post, or the launch) and flags it;
// the other waves end on the flag, or at their own limit.
template <int MIS, int COOP>
__global__ __launch_bounds__(kWave) void rx_service_kernel(SArgs s) {
  const int lane = threadIdx.x;
  const uint32_t w = blockIdx.x, W = gridDim.x;
  const uint32_t* mw = reinterpret_cast<const uint32_t*>(s.mail);
  uint32_t last = s.last;
  uint64_t t0 = wall_clock64();
  chain_init(lane); // any wave of the tier may complete a linked post
  for (;;) {
    const uint32_t v = lane <= (int)kExitFlag ? __hip_atomic_load(mw + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
    if (w != 0 && (uint32_t)__builtin_amdgcn_readlane(v, kExitFlag) == s.epoch) return; // wave 0 ended
    // the next post, k = last + 1, in its slot k & 1 -- and only there: a wave never passes over a post it may run on
    // (an earlier read of the other slot could be older than this one's)
    const uint32_t k = last + 1;
    const uint32_t b = (k & 1) * 16; // the slot's words: lanes b .. b + 15
    const uint32_t q = __builtin_amdgcn_readlane(v, b + 15);
    uint32_t x = q; // the check word over words 1-13 (svc_check)
#pragma unroll
    for (uint32_t i = 1; i <= 13; i++) x ^= (uint32_t)__builtin_amdgcn_readlane(v, b + i);
    const bool whole = (uint32_t)__builtin_amdgcn_readlane(v, b) == q && (uint32_t)__builtin_amdgcn_readlane(v, b + 14) == x;
    if (!whole || (int32_t)(q - k) < 0) { // post k is not there yet
      if (w == 0) {
        if (wall_clock64() - t0 > s.idle_ticks) { // no post for idle_ms: end, and say so
          if (lane == 0) {
            __hip_atomic_store(const_cast<uint32_t*>(mw) + kExitFlag, s.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(s.exit_word, s.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          return;
        }
        __builtin_amdgcn_s_sleep(1);
      } else {
        if (wall_clock64() - t0 > s.net_ticks) return; // a safety net: wave 0 always flags its end first
        for (uint32_t i = 0; i < s.poll_sleep; ++i) __builtin_amdgcn_s_sleep(1);
      }
      continue;
    }
    if (q != k) { // the slot already holds a later post: post k was complete without this wave, which was not one of
      last = k;   // its waves (the host reuses a slot only once its post is complete)
      t0 = wall_clock64();
      continue;
    }
    const uint32_t nw = __builtin_amdgcn_readlane(v, b + 1);
    if (nw == PN_SERVICE_STOP) return;
    last = k;
    const uint32_t fw = __builtin_amdgcn_readlane(v, b + 2);
    const uint32_t act = svc_active(nw & kPostN, fw & 0xffu, W + (fw >> 8));
    if (w < act) { // this wave runs on post k
      SVC_T(w, 0);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); // the frames the host wrote before the post
      SVC_T(w, 1);
      const KArgsAux a = svc_args(v, b, s, k);
      SVC_T(w, 5);
      const bool linked = a.aux != nullptr;
      svc_run<MIS, COOP>(a, (nw & kPostVerify) != 0, linked, w, act, k, s.done_words + w, lane);
      SVC_T(w, 6);
      if (act > kDoneWords || linked) {
        uint32_t* cw = s.done_words + kCountWords + (k & 1);
        if (act == 1) svc_finish<true>(a, svc_links(v, b), k, cw, lane);
        else svc_count<true>(&s.dev->count[k & 1][0], a, svc_links(v, b), act < W ? act : W, k, cw, lane);
      }
      SVC_T(w, 7);
    }
    t0 = wall_clock64();
  }
}

// The helper waves of a large post: waves kLatWaves + blockIdx.x of it, with the post's arguments from the host (the
// launch is issued with the post).  Their groups are theirs alone and nothing on the device waits for them: they run
// as soon as they are scheduled, even before wave 0 has taken the post, and end; the host counts the post done once
// their grid has ended (svc_post_done), and that end makes their records visible.
template <int MIS, int COOP>
__global__ __launch_bounds__(kWave) void rx_service_helper_kernel(KArgsAux a, uint32_t verify, uint32_t act) {
  svc_run<MIS, COOP, true>(a, verify != 0, false, kLatWaves + blockIdx.x, act, 0, nullptr, threadIdx.x);
}

template <int MIS>
void launch_svc(bool coop, uint32_t waves, const SArgs& a, hipStream_t s) {
  if (coop) hipLaunchKernelGGL((rx_service_kernel<MIS, 1>), dim3(waves), dim3(kWave), 0, s, a);
  else hipLaunchKernelGGL((rx_service_kernel<MIS, 0>), dim3(waves), dim3(kWave), 0, s, a);
}

template <int MIS>
void launch_helpers(bool coop, uint32_t helpers, const KArgsAux& a, uint32_t verify, uint32_t act, hipStream_t s) {
  if (coop) hipLaunchKernelGGL((rx_service_helper_kernel<MIS, 1>), dim3(helpers), dim3(kWave), 0, s, a, verify, act);
  else hipLaunchKernelGGL((rx_service_helper_kernel<MIS, 0>), dim3(helpers), dim3(kWave), 0, s, a, verify, act);
}
} // namespace

struct pn_service {
  pn_ctx* ctx = nullptr;
  hipStream_t stream = nullptr;        // the resident kernel (the latency tier)
  hipStream_t helper_stream = nullptr; // large posts' helper grids
  uint32_t stride = 0, frame_off = 0;
  uint32_t helpers_max = 0;            // helper waves of a large post: its total wave count less the tier's
  uint32_t post_helpers[2] = {0, 0};   // helper waves of the last two posts (a relaunch launches them again)
  hipEvent_t helper_ev[2] = {nullptr, nullptr}; // the end of each one's helper grid: its records are visible then
  uint64_t idle_ticks = 0, net_ticks = 0;
  SvcPost* mail = nullptr;    // the two slots and the exit flag's line: device memory the host writes through the
  bool mail_dev = false;      // large BAR (mail_dev), or pinned host memory; the host only ever stores to it
  uint32_t* words = nullptr;  // pinned host: [0, 64) the waves' done words, [kExitWord] exit (its own line)
  uint32_t post_words[2] = {0, 0}; // the last two posts (slot k & 1): the waves whose done words post k completes
                                   // through, or 0 for a counted post (its slot's count word)
  // the conn-table buffer each post captured (ctx->tbl_buf[b]): the last post that did, per buffer, so that
  // pn_set_conn_table waits for it before it overwrites or frees that buffer (svc_release_table)
  uint32_t tbl_post[2] = {0, 0};
  bool tbl_used[2] = {false, false};
  SvcDev* dev = nullptr;      // device
  u32x4* scratch = nullptr;   // device: the chain entries of linked posts, kLinkFrames x 2 per mailbox slot
  uint32_t seq = 0;           // last post issued
  uint32_t epoch = 0;         // launches so far (never 0: the exit flag's initial value)
  bool running = false;       // a launch that has not been seen to end
  bool coop = false;
};

namespace {
// Launch (or relaunch) the kernel; it starts waiting for post base + 1, base = the last completed post, so posts
// issued but not yet seen by an ended launch are taken by this one (they are still in their slots).
SArgs svc_sargs(const pn_service* v, uint32_t base) {
  SArgs a;
  a.mail = v->mail;
  a.scratch = v->scratch;
  a.done_words = v->words;
  a.exit_word = v->words + kExitWord;
  a.dev = v->dev;
  a.idle_ticks = v->idle_ticks;
  a.net_ticks = v->net_ticks;
  a.epoch = v->epoch;
  a.last = base;
  a.stride = v->stride;
  a.ipa_off = (v->frame_off + 14) & ~15u;
  a.avail = v->stride - v->frame_off;
  a.poll_sleep = v->mail_dev ? 1u : 16u; // polls of host memory cross PCIe: fewer of them
  return a;
}

// x86 store fence: the mailbox's stores out of the write-combining buffer, in order (device memory through the BAR
// is write-combined; for pinned host memory the fence costs little)
inline void host_sfence() { asm volatile("sfence" ::: "memory"); }

// Write post q into its slot.  Only stores: a read of device memory through the BAR would cost a PCIe round trip.
// Device memory (write-combined): the whole 64-B line as two 32-B non-temporal stores and one fence, so it leaves the
// write-combining buffer as one write (a read that still splits it fails the check word).  Pinned host memory, or a
// CPU without AVX: words 1-14 (the fields and the check word), a fence, then gen and seq, a fence.
void svc_publish(SvcPost* slot, const SvcPost& q, bool wc) {
  static const bool avx = __builtin_cpu_supports("avx");
  if (wc && avx) {
    asm volatile(
        "vmovdqu (%0), %%ymm0\n\t"
        "vmovdqu 32(%0), %%ymm1\n\t"
        "vmovntdq %%ymm0, (%1)\n\t"
        "vmovntdq %%ymm1, 32(%1)\n\t"
        "sfence\n\t"
        "vzeroupper"
        :
        : "r"(&q), "r"(slot)
        : "memory", "xmm0", "xmm1");
    return;
  }
  volatile uint32_t* d = reinterpret_cast<volatile uint32_t*>(slot);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&q);
  for (int i = 1; i <= 14; ++i) d[i] = w[i];
  host_sfence();
  d[0] = w[0];
  d[15] = w[15];
  host_sfence();
}

// the helper grid of large post k (its fields q), and the event its end completes: the post is done once both its
// resident waves' done word and the grid's end are
int svc_launch_helpers(pn_service* v, uint32_t k, uint32_t helpers, const SvcPost& q) {
  const SvcPost* p = &q;
  KArgsAux a;
  a.n = p->n & kPostN;
  a.fpw = p->fpw & 0xffu;
  a.max_conn = p->max_conn;
  a.frames = p->frames;
  a.out = p->out;
  a.tbl = p->tbl;
  a.mask = p->mask;
  a.n_entries = p->n_entries;
  a.stride = v->stride;
  a.ipa_off = (v->frame_off + 14) & ~15u;
  a.avail = v->stride - v->frame_off;
  a.offs = nullptr;
  a.aux = nullptr;
  const uint32_t verify = (p->n & kPostVerify) ? 1u : 0u, act = svc_active(a.n, a.fpw, kLatWaves + helpers);
  hipStream_t s = v->helper_stream;
  switch ((v->frame_off + 14) & 15) {
    case 0: launch_helpers<0>(v->coop, helpers, a, verify, act, s); break;
    case 2: launch_helpers<2>(v->coop, helpers, a, verify, act, s); break;
    case 4: launch_helpers<4>(v->coop, helpers, a, verify, act, s); break;
    case 6: launch_helpers<6>(v->coop, helpers, a, verify, act, s); break;
    case 8: launch_helpers<8>(v->coop, helpers, a, verify, act, s); break;
    case 10: launch_helpers<10>(v->coop, helpers, a, verify, act, s); break;
    case 12: launch_helpers<12>(v->coop, helpers, a, verify, act, s); break;
    default: launch_helpers<14>(v->coop, helpers, a, verify, act, s); break;
  }
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && !v->helper_ev[k & 1]) e = hipEventCreateWithFlags(&v->helper_ev[k & 1], hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(v->helper_ev[k & 1], s);
  if (e != hipSuccess) return hip_err(v->ctx, e, "pn_service: helper launch");
  return PN_OK;
}

int svc_launch(pn_service* v, uint32_t base) {
  pn_ctx* ctx = v->ctx;
  const SvcDev init{};
  hipError_t e = hipMemcpyAsync(v->dev, &init, sizeof(SvcDev), hipMemcpyHostToDevice, v->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(v->stream); // the previous launch has ended, the state is in place
  if (e != hipSuccess) return hip_err(ctx, e, "pn_service: device state");
  if (++v->epoch == 0) ++v->epoch;
  const SArgs a = svc_sargs(v, base);
  switch ((v->frame_off + 14) & 15) {
    case 0: launch_svc<0>(v->coop, kLatWaves, a, v->stream); break;
    case 2: launch_svc<2>(v->coop, kLatWaves, a, v->stream); break;
    case 4: launch_svc<4>(v->coop, kLatWaves, a, v->stream); break;
    case 6: launch_svc<6>(v->coop, kLatWaves, a, v->stream); break;
    case 8: launch_svc<8>(v->coop, kLatWaves, a, v->stream); break;
    case 10: launch_svc<10>(v->coop, kLatWaves, a, v->stream); break;
    case 12: launch_svc<12>(v->coop, kLatWaves, a, v->stream); break;
    default: launch_svc<14>(v->coop, kLatWaves, a, v->stream); break;
  }
  e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "pn_service: launch");
  v->running = true; // posts issued but not completed (still in their slots) run again on this launch (their helper
  return PN_OK;      // grids, independent of it, are not relaunched)
}

// post k's own waves are done (k one of the last two posts): every done word it completes through holds k (or later),
// one per wave it ran on or word 0 alone for a counted post, and its helper grid has ended
bool svc_post_ran(const pn_service* v, uint32_t k) {
  const uint32_t words = v->post_words[k & 1];
  if (words == 0 && (int32_t)(__atomic_load_n(v->words + kCountWords + (k & 1), __ATOMIC_ACQUIRE) - k) < 0) return false;
  for (uint32_t w = 0; w < words; ++w)
    if ((int32_t)(__atomic_load_n(v->words + w, __ATOMIC_ACQUIRE) - k) < 0) return false;
  if (v->post_helpers[k & 1] && hipEventQuery(v->helper_ev[k & 1]) != hipSuccess) return false; // (an error: not done)
  return true;
}

// post k is complete: it ran, and so did the post before it.  The waves take posts in order, but post k + 1 may run
// on fewer waves than post k and finish first; completion stays in post order (the contract, and what lets the host
// reuse post k's slot, counter and scratch for post k + 2).  Only the last two posts can be outstanding.
bool svc_post_done(const pn_service* v, uint32_t k) {
  if ((int32_t)(v->seq - k) >= 2) return true;
  if (!svc_post_ran(v, k)) return false;
  return k != v->seq || svc_post_ran(v, k - 1);
}

// the last completed post (posts complete in order)
uint32_t svc_done(const pn_service* v) {
  if (svc_post_done(v, v->seq)) return v->seq;
  return svc_post_done(v, v->seq - 1) ? v->seq - 1 : v->seq - 2;
}

bool svc_exited(const pn_service* v) { return __atomic_load_n(v->words + kExitWord, __ATOMIC_ACQUIRE) == v->epoch; }

void svc_free(pn_service* v) {
  if (v->ctx) {
    auto& l = v->ctx->services;
    l.erase(std::remove(l.begin(), l.end(), v), l.end());
  }
  if (v->mail) (void)(v->mail_dev ? hipFree(v->mail) : hipHostFree(v->mail));
  if (v->words) (void)hipHostFree(v->words);
  if (v->dev) (void)hipFree(v->dev);
  if (v->scratch) (void)hipFree(v->scratch);
  if (v->stream) (void)hipStreamDestroy(v->stream);
  if (v->helper_stream) (void)hipStreamDestroy(v->helper_stream);
  for (hipEvent_t ev : v->helper_ev)
    if (ev) (void)hipEventDestroy(ev);
  delete v;
}
} // namespace

// pn_set_conn_table is about to overwrite (or free) table buffer `buf`: every post of the ctx's services that captured
// it must be complete first.  Only one of the last two posts can still be running; an older one is done by
// construction (post k was issued only once post k - 2 was).
int pn_internal::svc_release_table(pn_ctx* ctx, int buf) {
  for (pn_service* v : ctx->services) {
    if (!v->tbl_used[buf]) continue;
    const uint32_t id = v->tbl_post[buf];
    if ((int32_t)(v->seq - id) < 2 && !svc_post_done(v, id)) {
      const int rc = pn_service_wait(v, id);
      if (rc) return rc;
    }
    v->tbl_used[buf] = false;
  }
  return PN_OK;
}

extern "C" {

int pn_service_open(pn_ctx* ctx, uint32_t slot_stride, uint32_t frame_off, uint32_t idle_ms, pn_service** out) {
  return pn_service_open_ex(ctx, slot_stride, frame_off, idle_ms, 0, out);
}

int pn_service_open_ex(pn_ctx* ctx, uint32_t slot_stride, uint32_t frame_off, uint32_t idle_ms, uint32_t large_waves,
                       pn_service** out) {
  if (!ctx || !out) return set_err(ctx, PN_EINVAL, "pn_service_open: ctx / out is NULL");
  *out = nullptr;
  if ((slot_stride & 15) || slot_stride > 65536 || (frame_off & 1) || slot_stride < frame_off + 96)
    return set_err(ctx, PN_EINVAL, "pn_service_open: slot_stride/frame_off violate the layout contract");
  if (idle_ms == 0 || idle_ms > 10000) return set_err(ctx, PN_EINVAL, "pn_service_open: idle_ms must be in [1, 10000]");
  if (large_waves && (large_waves < PN_SERVICE_WAVES || large_waves > PN_SERVICE_MAX_WAVES))
    return set_err(ctx, PN_EINVAL, "pn_service_open: large_waves must be 0 or in [PN_SERVICE_WAVES, PN_SERVICE_MAX_WAVES]");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  int khz = 0;
  e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device);
  if (e != hipSuccess || khz <= 0) return hip_err(ctx, e, "pn_service_open: wall clock rate");
  int cus = 0;
  e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device);
  if (e != hipSuccess || cus <= 0) return hip_err(ctx, e, "pn_service_open: CU count");
  pn_service* v = new pn_service();
  v->ctx = ctx;
  v->stride = slot_stride;
  v->frame_off = frame_off;
  // a large post: the latency tier plus helpers, enough waves to stream it at pn_classify's rate
  const uint32_t total = large_waves ? large_waves
                                     : std::max<uint32_t>(kLatWaves, std::min<uint32_t>(PN_SERVICE_MAX_WAVES,
                                                                                      (uint32_t)cus * PN_SERVICE_WAVES_PER_CU));
  v->helpers_max = total - kLatWaves;
  v->idle_ticks = (uint64_t)khz * idle_ms;
  v->net_ticks = v->idle_ticks + (v->idle_ticks >> 1) + (uint64_t)khz * kNetLimitMs;
  // the cooperative window needs a 16-B chunk before it inside the slot (frame_off >= 2); the frames' 16-B
  // alignment is checked per post
  v->coop = (slot_stride % 16) == 0 && ((frame_off + 14) & ~15u) >= 16;
  // the mailbox in uncached device memory when the host can store to it through a large BAR
  int large_bar = 0;
  if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, ctx->device) != hipSuccess) large_bar = 0;
  v->mail_dev = large_bar != 0 && std::getenv("PN_SERVICE_HOST_MAILBOX") == nullptr;
  if (v->mail_dev && hipExtMallocWithFlags((void**)&v->mail, kMailBytes, hipDeviceMallocUncached) != hipSuccess) {
    (void)hipGetLastError(); // no uncached device memory: the mailbox in pinned host memory
    v->mail = nullptr;
    v->mail_dev = false;
  }
  if ((e = hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&v->helper_stream, hipStreamNonBlocking)) != hipSuccess ||
      (!v->mail && (e = hipHostMalloc((void**)&v->mail, kMailBytes, hipHostMallocDefault)) != hipSuccess) ||
      (e = hipHostMalloc((void**)&v->words, kWordsBytes, hipHostMallocDefault)) != hipSuccess ||
      (e = hipMalloc((void**)&v->dev, sizeof(SvcDev))) != hipSuccess ||
      (e = hipMalloc((void**)&v->scratch, sizeof(u32x4) * 2 * 2 * kLinkFrames)) != hipSuccess) {
    const int rc = hip_err(ctx, e, "pn_service_open: allocation");
    svc_free(v);
    return rc;
  }
  // The post counter's start: 0, or PN_SERVICE_FIRST_POST from the environment (tests start it just below 2^32 to
  // run the counter's wrap).  The done words and both slots hold it: neither slot reads as post first + 1 or + 2.
  uint32_t first = 0;
  if (const char* env = std::getenv("PN_SERVICE_FIRST_POST")) first = (uint32_t)std::strtoull(env, nullptr, 0);
  std::memset(v->words, 0, kWordsBytes);
  for (uint32_t w = 0; w < kDoneWords + 2; ++w) v->words[w] = first; // the done and count words
  {
    SvcPost q{};
    q.gen = q.seq = first;
    q.check = ~svc_check(&q, first); // not a whole post either (and `first` is no post after the start)
    for (int i = 0; i < 2; ++i) svc_publish(v->mail + i, q, v->mail_dev);
    volatile uint32_t* flag = reinterpret_cast<volatile uint32_t*>(v->mail) + kExitFlag;
    *flag = 0u; // no launch has epoch 0
    host_sfence();
  }
  v->seq = first;
  const int rc = svc_launch(v, first);
  if (rc) {
    svc_free(v);
    return rc;
  }
  ctx->services.push_back(v);
  *out = v;
  return PN_OK;
}

int pn_service_post(pn_service* v, const void* frames, uint32_t n, void* results, uint32_t* post_id) {
  return pn_service_post_linked(v, frames, n, results, nullptr, post_id);
}

int pn_service_post_linked(pn_service* v, const void* frames, uint32_t n, void* results, uint16_t* links,
                           uint32_t* post_id) {
  if (!v) return set_err(nullptr, PN_EINVAL, "pn_service_post: service is NULL");
  pn_ctx* ctx = v->ctx;
  if (!ctx->tbl_dev) return set_err(ctx, PN_ENOTABLE, "pn_service_post: no conn table (call pn_set_conn_table)");
  if (n == 0 || n > PN_SERVICE_MAX_FRAMES || !frames || !results)
    return set_err(ctx, PN_EINVAL, "pn_service_post: n must be in [1, PN_SERVICE_MAX_FRAMES], buffers set");
  if (((uintptr_t)frames & 15) || ((uintptr_t)results & 15))
    return set_err(ctx, PN_EINVAL, "pn_service_post: frames/results must be 16-byte aligned");
  if (links && (n > PN_LINK_MAX_FRAMES || ((uintptr_t)links & 1)))
    return set_err(ctx, PN_EINVAL, "pn_service_post_linked: n must be <= PN_LINK_MAX_FRAMES, links 2-byte aligned");
  // at most two posts outstanding: post k reuses the slot of post k - 2, which must be done
  const uint32_t done = svc_done(v);
  if ((int32_t)(v->seq - done) >= 2) return set_err(ctx, PN_EINVAL, "pn_service_post: two posts already outstanding");
  if (v->running && svc_exited(v)) v->running = false; // ended: idle
  if (!v->running) {
    const int rc = svc_launch(v, done);
    if (rc) return rc;
  }
  const uint32_t k = v->seq + 1;
  // the post's line (svc_publish): the slot still holds post k - 2 (complete), so until gen and seq both read k it is
  // not post k; and should a wave's read of the line be split into pieces read at different times, a mix of two
  // posts' words fails the check and the wave reads the slot again
  const bool verify = ctx->verify_tcp;
  SvcPost q{};
  q.n = n | (verify ? kPostVerify : 0u) | (links ? kPostLinks : 0u);
  q.max_conn = ctx->max_conn;
  q.frames = (const uint8_t*)frames;
  q.out = (pn_result*)results;
  q.tbl = ctx->tbl_dev;
  q.links = links;
  q.mask = (uint32_t)ctx->mask;
  q.n_entries = ctx->n_entries;
  const uint32_t fpw = svc_fpw(n, verify), helpers = svc_helpers(n, v->helpers_max);
  q.fpw = fpw | helpers << 8;
  const uint32_t act = svc_active(n, fpw, kLatWaves + helpers);
  // a large post's helpers first (nothing waits for them on the device): should the launch fail, nothing was posted
  if (helpers) {
    const int rc = svc_launch_helpers(v, k, helpers, q);
    if (rc) return rc;
  }
  v->post_helpers[k & 1] = helpers;
  v->post_words[k & 1] = (act <= kDoneWords && !links) ? act : 0u; // else counted: its slot's count word (svc_finish)
  v->tbl_post[ctx->cur] = k; // pn_set_conn_table waits for this post before it reuses the buffer
  v->tbl_used[ctx->cur] = true;
  q.check = svc_check(&q, k);
  q.gen = q.seq = k;
  svc_publish(v->mail + (k & 1), q, v->mail_dev);
  v->seq = k;
  if (post_id) *post_id = k;
  return PN_OK;
}

int pn_service_wait(pn_service* v, uint32_t post_id) {
  if (!v) return set_err(nullptr, PN_EINVAL, "pn_service_wait: service is NULL");
  if (post_id == 0 || (int32_t)(post_id - v->seq) > 0 || (int32_t)(v->seq - post_id) >= 2)
    post_id = v->seq; // 0 (or an id not among the last two posts): the last post
  const uint32_t k = post_id;
  const auto t_start = std::chrono::steady_clock::now();
  for (uint64_t i = 1;; ++i) {
    if (svc_post_done(v, k)) return PN_OK;
    if ((i & 4095) == 0) {
      if (std::chrono::steady_clock::now() - t_start > std::chrono::seconds(10))
        return set_err(v->ctx, PN_EHIP, "pn_service_wait: no completion within 10 s");
      // the launch ended by itself (no post for idle_ms) before it saw this one: relaunch, it takes the pending
      // posts (the device state starts at the last completed one)
      if (svc_exited(v)) {
        const uint32_t done = svc_done(v);
        if ((int32_t)(done - k) >= 0) return PN_OK;
        v->running = false;
        const int rc = svc_launch(v, done);
        if (rc) return rc;
        continue;
      }
      const hipError_t q = hipStreamQuery(v->stream);
      if (q != hipErrorNotReady && q != hipSuccess) return hip_err(v->ctx, q, "pn_service_wait: the service kernel failed");
      if (q == hipSuccess && !svc_post_done(v, k) && !svc_exited(v))
        return set_err(v->ctx, PN_EHIP, "pn_service_wait: the service kernel ended without completing the post");
    }
  }
}

int pn_service_close(pn_service* v) {
  if (!v) return PN_OK;
  pn_ctx* ctx = v->ctx;
  // the outstanding posts first (a launch that ended before it took them is relaunched), then the stop
  int rc = svc_post_done(v, v->seq) ? PN_OK : pn_service_wait(v, 0);
  if (v->running && !svc_exited(v)) {
    const uint32_t k = v->seq + 1;
    SvcPost q{};
    q.n = PN_SERVICE_STOP;
    v->post_words[k & 1] = 0;
    v->post_helpers[k & 1] = 0;
    q.check = svc_check(&q, k);
    q.gen = q.seq = k;
    svc_publish(v->mail + (k & 1), q, v->mail_dev);
    v->seq = k;
  }
  hipError_t e = hipStreamSynchronize(v->stream); // the kernel ends at the stop or its idle limit
  if (e == hipSuccess) e = hipStreamSynchronize(v->helper_stream); // helpers end on the stop
  if (e != hipSuccess && rc == PN_OK) rc = hip_err(ctx, e, "pn_service_close");
  svc_free(v);
  return rc;
}

} // extern "C"

#ifdef PN_SVC_TRACE
// measurement build only: where the service kernels store their step clocks (64 waves x 8 u64, pinned host memory);
// set before pn_service_open
extern "C" int pn_svc_trace_set(uint64_t* host_buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_svc_trace), &host_buf, sizeof host_buf) == hipSuccess ? PN_OK : PN_EHIP;
}
#endif
