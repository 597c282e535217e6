// rmx_comd.cpp — see rmx_comd.h.  Reads the ELF section table, the NT_AMDGPU_METADATA note and its MessagePack
// document (.amdhsa.kernels: .symbol, .args[].offset / .size / .value_kind) with its own bounded reader.
#include "rmx_comd.h"

#include <elf.h>

#include <cstring>
#include <vector>

namespace rmx {
namespace {

struct HiddenSlot {
  const char* kind;
  uint32_t off, size;  // relative to the hidden base
};
// every hidden argument the queue provides (rmx_queue.cpp write_kernargs; the remainders and global offsets as zeros)
constexpr HiddenSlot kHidden[] = {
    {"hidden_block_count_x", 0, 4},    {"hidden_block_count_y", 4, 4},    {"hidden_block_count_z", 8, 4},
    {"hidden_group_size_x", 12, 2},    {"hidden_group_size_y", 14, 2},    {"hidden_group_size_z", 16, 2},
    {"hidden_remainder_x", 18, 2},     {"hidden_remainder_y", 20, 2},     {"hidden_remainder_z", 22, 2},
    {"hidden_global_offset_x", 40, 8}, {"hidden_global_offset_y", 48, 8}, {"hidden_global_offset_z", 56, 8},
    {"hidden_grid_dims", 64, 2},       {"hidden_dynamic_lds_size", 120, 4},
};
static_assert(kHidden[13].off + kHidden[13].size == kHiddenUsed, "the last hidden argument the queue writes");

// A MessagePack reader over one buffer: typed reads return false (and set bad) on a type or bounds mismatch.
struct Mp {
  const unsigned char* p;
  const unsigned char* end;
  bool bad = false;
  bool need(size_t n) {
    if ((size_t)(end - p) < n) bad = true;
    return !bad;
  }
  uint64_t be(int n) {  // big-endian unsigned of n bytes (bounds checked by the caller)
    uint64_t v = 0;
    for (int i = 0; i < n; ++i) v = v << 8 | p[i];
    p += n;
    return v;
  }
  int64_t len(unsigned fix_tag, unsigned fix_mask, unsigned tag16) {  // map / array header: element count or -1
    if (!need(1)) return -1;
    const unsigned c = *p;
    if ((c & ~fix_mask) == fix_tag) {
      ++p;
      return c & fix_mask;
    }
    if (c == tag16 && need(3)) return ++p, (int64_t)be(2);
    if (c == tag16 + 1 && need(5)) return ++p, (int64_t)be(4);
    bad = true;
    return -1;
  }
  int64_t map_len() { return len(0x80, 0x0F, 0xDE); }
  int64_t arr_len() { return len(0x90, 0x0F, 0xDC); }
  bool str(std::string* out) {
    if (!need(1)) return false;
    const unsigned c = *p;
    uint64_t n;
    if ((c & 0xE0) == 0xA0) n = c & 31, ++p;
    else if (c == 0xD9 && need(2)) ++p, n = be(1);
    else if (c == 0xDA && need(3)) ++p, n = be(2);
    else if (c == 0xDB && need(5)) ++p, n = be(4);
    else return bad = true, false;
    if (!need(n)) return false;
    out->assign(reinterpret_cast<const char*>(p), (size_t)n);
    p += n;
    return true;
  }
  bool uint(uint64_t* out) {  // a non-negative integer of any width
    if (!need(1)) return false;
    const unsigned c = *p;
    if (c <= 0x7F) return *out = c, ++p, true;
    static const int w[4] = {1, 2, 4, 8};
    if (c >= 0xCC && c <= 0xD3) {
      const int n = w[(c - 0xCC) & 3];
      if (!need(1 + (size_t)n)) return false;
      ++p;
      *out = be(n);
      if (c >= 0xD0 && (*out >> (8 * n - 1) & 1)) return bad = true, false;  // a negative signed value
      return true;
    }
    return bad = true, false;
  }
  bool skip(int depth = 0) {  // any value
    if (!need(1) || depth > 32) return bad = true, false;
    const unsigned c = *p;
    if (c <= 0x7F || c >= 0xE0 || c == 0xC0 || c == 0xC2 || c == 0xC3) return ++p, true;
    if ((c & 0xE0) == 0xA0 || (c >= 0xD9 && c <= 0xDB)) {
      std::string s;
      return str(&s);
    }
    if ((c & 0xF0) == 0x80 || c == 0xDE || c == 0xDF) {
      const int64_t n = map_len();
      for (int64_t i = 0; i < n && !bad; ++i) skip(depth + 1), skip(depth + 1);
      return !bad;
    }
    if ((c & 0xF0) == 0x90 || c == 0xDC || c == 0xDD) {
      const int64_t n = arr_len();
      for (int64_t i = 0; i < n && !bad; ++i) skip(depth + 1);
      return !bad;
    }
    size_t body;
    switch (c) {
      case 0xC4: case 0xC5: case 0xC6: {  // bin 8/16/32
        const int n = 1 << (c - 0xC4);
        if (!need(1 + (size_t)n)) return false;
        ++p;
        body = (size_t)be(n);
        break;
      }
      case 0xC7: case 0xC8: case 0xC9: {  // ext 8/16/32: length, type byte
        const int n = 1 << (c - 0xC7);
        if (!need(1 + (size_t)n)) return false;
        ++p;
        body = (size_t)be(n) + 1;
        break;
      }
      case 0xCA: ++p, body = 4; break;
      case 0xCB: ++p, body = 8; break;
      case 0xCC: case 0xCD: case 0xCE: case 0xCF: case 0xD0: case 0xD1: case 0xD2: case 0xD3:
        body = (size_t)1 << (c & 3), ++p;
        break;
      case 0xD4: case 0xD5: case 0xD6: case 0xD7: case 0xD8:  // fixext 1..16: type byte + body
        body = 1 + ((size_t)1 << (c - 0xD4)), ++p;
        break;
      default: return bad = true, false;
    }
    if (!need(body)) return false;
    p += body;
    return true;
  }
};

struct ArgMeta {
  uint64_t offset = 0, size = 0;
  std::string kind;
};

// "" when the queue can dispatch a step kernel with these arguments, else why not
std::string check_step_args(const std::vector<ArgMeta>& args, const CoLayout& L) {
  const uint64_t kExplicit[][2] = {{0, 4}, {4, 4}, {8, 8}, {16, 8}, {24, 8}, {32, 8}, {40, 8}, {48, 8},
                                   {L.fp_offset, L.fp_size}};
  size_t n_explicit = 0;
  for (const ArgMeta& a : args) {
    if (a.kind.compare(0, 7, "hidden_") != 0) {
      if (n_explicit >= sizeof(kExplicit) / sizeof(kExplicit[0]) || a.offset != kExplicit[n_explicit][0] ||
          a.size != kExplicit[n_explicit][1])
        return "explicit argument " + std::to_string(n_explicit) + " is not StepArgs' layout";
      ++n_explicit;
      continue;
    }
    if (a.kind == "hidden_none") continue;  // padding the runtime leaves alone
    const HiddenSlot* s = nullptr;
    for (const HiddenSlot& h : kHidden)
      if (a.kind == h.kind) s = &h;
    if (!s) return "hidden argument " + a.kind + " is not written by the queue";
    if (a.offset != L.hidden_base + s->off || a.size != s->size)
      return a.kind + " at offset " + std::to_string(a.offset) + " (the queue writes it at " +
             std::to_string(L.hidden_base + s->off) + ")";
  }
  if (n_explicit != sizeof(kExplicit) / sizeof(kExplicit[0])) return "explicit arguments are not StepArgs";
  return "";
}

void parse_kernels(Mp& m, CoCheck& out, const CoLayout& L) {
  const int64_t nk = m.arr_len();
  for (int64_t k = 0; k < nk && !m.bad; ++k) {
    std::string symbol, key;
    std::vector<ArgMeta> args;
    const int64_t nf = m.map_len();
    for (int64_t f = 0; f < nf && !m.bad; ++f) {
      if (!m.str(&key)) break;
      if (key == ".symbol") {
        m.str(&symbol);
      } else if (key == ".args") {
        const int64_t na = m.arr_len();
        for (int64_t i = 0; i < na && !m.bad; ++i) {
          ArgMeta a;
          const int64_t nm = m.map_len();
          for (int64_t j = 0; j < nm && !m.bad; ++j) {
            if (!m.str(&key)) break;
            if (key == ".offset") m.uint(&a.offset);
            else if (key == ".size") m.uint(&a.size);
            else if (key == ".value_kind") m.str(&a.kind);
            else m.skip();
          }
          args.push_back(a);
        }
      } else {
        m.skip();
      }
    }
    if (m.bad || symbol.find("step_fast_kernel") == std::string::npos) continue;
    ++out.n_step;
    const std::string why = check_step_args(args, L);
    if (!why.empty()) out.refused.emplace(symbol, why);
  }
}

}  // namespace

CoCheck check_code_object(const unsigned char* co, size_t bytes, const CoLayout& L) {
  CoCheck out;
  Elf64_Ehdr eh;
  if (bytes < sizeof(eh)) return out.err = "not an ELF object", out;
  std::memcpy(&eh, co, sizeof(eh));
  if (std::memcmp(eh.e_ident, ELFMAG, SELFMAG) != 0 || eh.e_ident[EI_CLASS] != ELFCLASS64 ||
      eh.e_shentsize != sizeof(Elf64_Shdr) || eh.e_shoff > bytes ||
      (bytes - eh.e_shoff) / sizeof(Elf64_Shdr) < eh.e_shnum)
    return out.err = "not a 64-bit ELF object", out;
  bool found = false;
  for (unsigned s = 0; s < eh.e_shnum; ++s) {
    Elf64_Shdr sh;
    std::memcpy(&sh, co + eh.e_shoff + (size_t)s * sizeof(sh), sizeof(sh));
    if (sh.sh_type != SHT_NOTE || sh.sh_offset > bytes || sh.sh_size > bytes - sh.sh_offset) continue;
    size_t o = (size_t)sh.sh_offset;
    const size_t e = o + (size_t)sh.sh_size;
    while (e - o >= sizeof(Elf64_Nhdr)) {
      Elf64_Nhdr nh;
      std::memcpy(&nh, co + o, sizeof(nh));
      const size_t name_at = o + sizeof(nh), desc_at = name_at + (((size_t)nh.n_namesz + 3) & ~(size_t)3);
      if (desc_at > e || nh.n_descsz > e - desc_at) break;
      if (nh.n_type == 32 /* NT_AMDGPU_METADATA */ && nh.n_namesz == 7 &&
          std::memcmp(co + name_at, "AMDGPU", 7) == 0) {
        Mp m{co + desc_at, co + desc_at + nh.n_descsz};
        std::string key;
        const int64_t n = m.map_len();
        for (int64_t i = 0; i < n && !m.bad; ++i) {
          if (!m.str(&key)) break;
          if (key == "amdhsa.kernels") parse_kernels(m, out, L), found = true;
          else m.skip();
        }
        if (m.bad) return out.err = "malformed AMDGPU metadata", out;
      }
      // the next note: a descriptor that ends the section without its padding ends the walk (the padded end may lie
      // past the section and the buffer)
      const size_t next = desc_at + (((size_t)nh.n_descsz + 3) & ~(size_t)3);
      if (next > e) break;
      o = next;
    }
  }
  if (!found) out.err = "no amdhsa.kernels metadata";
  return out;
}


}  // namespace rmx
