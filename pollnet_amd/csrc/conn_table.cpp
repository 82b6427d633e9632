// Host-side connection table: the control plane that produces the read-only
// snapshot the RX kernel probes.  Same data contract as efvitcp's Core:
//   ConnHashEntry{u64 key; u32 conn_id} (Core.h:178-182), 16 B with padding,
//   MaxTableSize = 1 << (1 + getMSB(MaxConn + MaxTW)) (Core.h:235),
//   TotalTableSize = MaxTableSize + MaxConn + MaxTW (Core.h:236),
//   initial tbl_mask = min(MaxTableSize, 128) - 1 (Core.h:322),
//   ordered (sorted-run) linear probing that spills past tbl_mask instead of
//   wrapping (findConnEntry Core.h:558-562, addConnEntry :566-576,
//   delConnEntry :578-605, tryExpandConnTbl :650-682).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <new>
#include <utility>
#include <vector>

#include "../../include/pollnet_amd.h"

namespace {

constexpr int msb_count(uint32_t n) { return n == 0 ? 0 : msb_count(n >> 1) + 1; } // getMSB, Core.h:174

struct ConnTable {
  std::vector<pn_conn_entry> tbl;
  uint64_t mask = 0;
  uint32_t max_conn = 0, max_tw = 0, size = 0;
  uint32_t repairs = 0;
  bool literal = false; // PN_TABLE_REFERENCE_LITERAL: keep tryExpandConnTbl's result as it is

  bool init(uint32_t mc, uint32_t mtw, bool lit) {
    literal = lit;
    max_conn = mc;
    max_tw = mtw;
    uint64_t max_tbl = 1ull << (1 + msb_count(mc + mtw));
    if (max_tbl > (1ull << 28)) return false;
    tbl.assign(max_tbl + mc + mtw, pn_conn_entry{PN_EMPTY_KEY, 0, 0});
    mask = std::min<uint64_t>(max_tbl, 128) - 1;
    size = 0;
    return true;
  }

  // Ordered probe: first entry whose key is >= `key`.  Runs are sorted and an
  // EmptyKey (1<<63, above every 48-bit key) ends them; bounded at the array end.
  uint32_t find(uint64_t key) const {
    uint64_t e = key & mask;
    const uint64_t n = tbl.size();
    while (e < n && tbl[e].key < key) ++e;
    return (uint32_t)e;
  }

  // Ordered insertion of a key known to be absent (the addConnEntry loop).
  void insert_sorted(uint64_t key, uint32_t conn_id) {
    uint32_t e = find(key);
    while (tbl[e].key != PN_EMPTY_KEY) {
      std::swap(tbl[e].key, key);
      std::swap(tbl[e].conn_id, conn_id);
      while (tbl[++e].key < key) {
      }
    }
    tbl[e].key = key;
    tbl[e].conn_id = conn_id;
  }

  void expand() {
    if ((uint64_t)size * 2 <= mask) return;
    // The reference's in-place rehash (Core.h:656-678) assumes every findConnEntry
    // during the rehash stops on the entry itself or on an empty slot (its debug
    // build exits otherwise, Core.h:665-669).  That fails when a spill run past the
    // old mask is rehashed after first-segment keys already moved into the upper
    // half: the larger key found is swapped into the spill region with the wrong
    // conn_id and becomes unreachable.  We run the reference's rehash verbatim and,
    // only if that condition fires, rebuild the table from a snapshot instead
    // (ordered hashing has one canonical layout per key set, which is what the
    // reference produces whenever its rehash is well-defined).  In reference-literal
    // mode the table keeps exactly what the reference's rehash leaves, stranded keys
    // included, so that records match the reference bit for bit under such histories.
    std::vector<pn_conn_entry> saved;
    saved.reserve(size);
    for (const auto& x : tbl)
      if (x.key != PN_EMPTY_KEY) saved.push_back(x);
    bool broken = false;
    uint64_t end = mask + 1;
    mask = mask * 2 + 1;
    uint64_t new_end = mask + 1;
    // the spill run past the old mask moves past the new mask first
    while (tbl[end].key != PN_EMPTY_KEY) std::swap(tbl[new_end++], tbl[end++]);
    const uint64_t end_cnt = new_end - (mask + 1);
    auto rehash = [&](uint64_t e, uint64_t cnt) {
      for (; cnt; ++e) {
        if (tbl[e].key == PN_EMPTY_KEY) continue;
        uint32_t ne = find(tbl[e].key);
        if (tbl[ne].key != tbl[e].key && tbl[ne].key != PN_EMPTY_KEY) broken = true;
        std::swap(tbl[e].key, tbl[ne].key);
        tbl[ne].conn_id = tbl[e].conn_id;
        --cnt;
      }
    };
    rehash(0, size - end_cnt);
    rehash(mask + 1, end_cnt);
    if (broken && !literal) {
      ++repairs;
      for (auto& x : tbl) x = pn_conn_entry{PN_EMPTY_KEY, 0, 0};
      for (const auto& x : saved) insert_sorted(x.key, x.conn_id);
    }
  }

  int add(uint64_t key, uint32_t conn_id) {
    uint32_t e = find(key);
    if (e < tbl.size() && tbl[e].key == key) return PN_EINVAL;
    if (size >= max_conn + max_tw) return PN_EFULL;
    ++size; // callers bump conn_cnt/tw_cnt before addConnEntry (TcpServer.h:88-89)
    // insertion keeps each run sorted: carry the larger key forward
    insert_sorted(key, conn_id);
    expand();
    return PN_OK;
  }

  int del(uint64_t key) {
    uint32_t e = find(key);
    if (e >= tbl.size() || tbl[e].key != key) return PN_ENOENT;
    --size;
    // backward-shift: pull later run members whose home slot is <= the hole
    for (;;) {
      uint32_t next = e + 1;
      while ((tbl[next].key & mask) > e) ++next;
      if (tbl[next].key == PN_EMPTY_KEY) break;
      tbl[e] = tbl[next];
      e = next;
    }
    tbl[e].key = PN_EMPTY_KEY;
    return PN_OK;
  }
};

} // namespace

struct pn_conn_table {
  ConnTable t;
};

extern "C" {

uint64_t pn_conn_hash_key(uint32_t ip_be, uint16_t port_be) {
  // connHashKey (Core.h:167-172): remote ip (host order) << 15 | low 15 port bits,
  // port msb moved to bit 47 ("ephemeral ports have the msb set").
  uint64_t ip = __builtin_bswap32(ip_be);
  uint64_t p = __builtin_bswap16(port_be);
  return (ip << 15) | (p & 0x7fff) | ((p & 0x8000) << 32);
}

int pn_table_create(uint32_t max_conn_cnt, uint32_t max_tw_cnt, pn_conn_table** out) {
  return pn_table_create_ex(max_conn_cnt, max_tw_cnt, 0, out);
}

int pn_table_create_ex(uint32_t max_conn_cnt, uint32_t max_tw_cnt, uint32_t flags, pn_conn_table** out) {
  if (!out || max_conn_cnt == 0 || (flags & ~PN_TABLE_REFERENCE_LITERAL)) return PN_EINVAL;
  auto* t = new (std::nothrow) pn_conn_table();
  if (!t) return PN_ENOMEM;
  if (!t->t.init(max_conn_cnt, max_tw_cnt, flags & PN_TABLE_REFERENCE_LITERAL)) {
    delete t;
    return PN_EINVAL;
  }
  *out = t;
  return PN_OK;
}

void pn_table_destroy(pn_conn_table* t) { delete t; }

int pn_table_find(const pn_conn_table* t, uint64_t key, uint32_t* entry_idx, int* hit, uint32_t* conn_id) {
  if (!t) return PN_EINVAL;
  uint32_t e = t->t.find(key);
  bool h = e < t->t.tbl.size() && t->t.tbl[e].key == key;
  if (entry_idx) *entry_idx = e;
  if (hit) *hit = h;
  if (conn_id) *conn_id = h ? t->t.tbl[e].conn_id : PN_MISS;
  return PN_OK;
}

int pn_table_add(pn_conn_table* t, uint64_t key, uint32_t conn_id) {
  if (!t || key >= PN_EMPTY_KEY) return PN_EINVAL;
  return t->t.add(key, conn_id);
}

int pn_table_del(pn_conn_table* t, uint64_t key) {
  if (!t) return PN_EINVAL;
  return t->t.del(key);
}

int pn_table_set_conn_id(pn_conn_table* t, uint64_t key, uint32_t conn_id) {
  if (!t) return PN_EINVAL;
  uint32_t e = t->t.find(key);
  if (e >= t->t.tbl.size() || t->t.tbl[e].key != key) return PN_ENOENT;
  t->t.tbl[e].conn_id = conn_id;
  return PN_OK;
}

const pn_conn_entry* pn_table_entries(const pn_conn_table* t, uint32_t* n_entries, uint64_t* tbl_mask) {
  if (!t) return nullptr;
  if (n_entries) *n_entries = (uint32_t)t->t.tbl.size();
  if (tbl_mask) *tbl_mask = t->t.mask;
  return t->t.tbl.data();
}

uint32_t pn_table_max_conn_cnt(const pn_conn_table* t) { return t ? t->t.max_conn : 0; }
uint32_t pn_table_size(const pn_conn_table* t) { return t ? t->t.size : 0; }
uint32_t pn_table_repairs(const pn_conn_table* t) { return t ? t->t.repairs : 0; }
uint32_t pn_table_flags(const pn_conn_table* t) { return t && t->t.literal ? PN_TABLE_REFERENCE_LITERAL : 0u; }

} // extern "C"
