// Native caption tokenizer core (SURVEY D23 / §2.3 "tokenizers (Rust)"): the reference tokenizes every
// caption with T5TokenizerFast (reference task.py:58, data.py:24, inference/run_inference.py:47,81) -- a
// SentencePiece unigram model behind HuggingFace's Rust `tokenizers`. This header re-implements that
// pipeline in C++ with no Python dependency:
//
//   raw text -> split out added/special tokens -> normalizers (SentencePiece precompiled charsmap,
//   strip, replace, ASCII lowercase) -> pre-tokenizers (whitespace split, metaspace) -> unigram Viterbi
//   (best-scoring segmentation, unknown characters scored min_score - 10 and fused) -> ids
//   -> truncation + template post-processing (append </s>).
//
// Behaviour follows the observable semantics of the library (tie-breaking, unknown-run fusing,
// metaspace prepend schemes, truncation keeping room for the appended special tokens); parity is
// tested against `tokenizers` / `transformers` on locally trained SentencePiece models
// (tests/test_tokenizer_cpu.py). Grapheme clusters for the charsmap lookup are approximated as a base
// code point followed by combining marks / joiners / variation selectors.
#pragma once

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <regex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace dalle_tok {

// ---------------------------------------------------------------------------------------------
// UTF-8 helpers
// ---------------------------------------------------------------------------------------------
inline int utf8_len(unsigned char c) {
  if (c < 0x80) return 1;
  if ((c >> 5) == 0x6) return 2;
  if ((c >> 4) == 0xE) return 3;
  if ((c >> 3) == 0x1E) return 4;
  return 1;  // invalid lead byte: treat as one byte
}

inline uint32_t decode_cp(const std::string& s, size_t i, int n) {
  const unsigned char* p = reinterpret_cast<const unsigned char*>(s.data()) + i;
  switch (n) {
    case 1: return p[0];
    case 2: return ((p[0] & 0x1F) << 6) | (p[1] & 0x3F);
    case 3: return ((p[0] & 0x0F) << 12) | ((p[1] & 0x3F) << 6) | (p[2] & 0x3F);
    default: return ((p[0] & 0x07) << 18) | ((p[1] & 0x3F) << 12) | ((p[2] & 0x3F) << 6) | (p[3] & 0x3F);
  }
}

inline bool is_unicode_space(uint32_t c) {
  return c == ' ' || (c >= 0x09 && c <= 0x0D) || c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) ||
         c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}

// continues the previous grapheme cluster (approximation of UAX #29 extend / ZWJ / spacing marks)
inline bool is_extender(uint32_t c) {
  return (c >= 0x0300 && c <= 0x036F) || (c >= 0x0483 && c <= 0x0489) || (c >= 0x0591 && c <= 0x05BD) ||
         (c >= 0x0610 && c <= 0x061A) || (c >= 0x064B && c <= 0x065F) || (c >= 0x0900 && c <= 0x0903) ||
         (c >= 0x093A && c <= 0x094F) || (c >= 0x0E31 && c <= 0x0E3A && c != 0x0E32 && c != 0x0E33) ||
         (c >= 0x0E47 && c <= 0x0E4E) || (c >= 0x1AB0 && c <= 0x1AFF) || (c >= 0x1DC0 && c <= 0x1DFF) ||
         c == 0x200C || c == 0x200D || (c >= 0x20D0 && c <= 0x20FF) || (c >= 0x3099 && c <= 0x309A) ||
         (c >= 0xFE00 && c <= 0xFE0F) || (c >= 0xFE20 && c <= 0xFE2F) || (c >= 0x1F3FB && c <= 0x1F3FF) ||
         (c >= 0xE0100 && c <= 0xE01EF);
}

// ---------------------------------------------------------------------------------------------
// SentencePiece precompiled charsmap: [u32 trie bytes][darts-clone double array][NUL-separated outputs]
// ---------------------------------------------------------------------------------------------
class Charsmap {
 public:
  Charsmap() = default;
  explicit Charsmap(const std::string& blob) {
    if (blob.size() < 4) throw std::runtime_error("charsmap: blob too short");
    uint32_t trie_bytes;
    std::memcpy(&trie_bytes, blob.data(), 4);
    if (trie_bytes % 4 || 4 + size_t(trie_bytes) > blob.size()) throw std::runtime_error("charsmap: bad trie size");
    units_.resize(trie_bytes / 4);
    std::memcpy(units_.data(), blob.data() + 4, trie_bytes);
    outputs_ = blob.substr(4 + trie_bytes);
  }
  bool empty() const { return units_.empty(); }

  // first (shortest) prefix of s[b:e) present in the map -> its replacement
  bool transform(const char* s, size_t n, std::string* out) const {
    if (units_.empty()) return false;
    size_t pos = 0;
    uint32_t unit = units_[0];
    pos ^= offset(unit);
    for (size_t i = 0; i < n; ++i) {
      unsigned char c = static_cast<unsigned char>(s[i]);
      if (c == 0) break;
      pos ^= c;
      if (pos >= units_.size()) return false;
      unit = units_[pos];
      if (label(unit) != c) return false;
      pos ^= offset(unit);
      if (has_leaf(unit)) {
        if (pos >= units_.size()) return false;
        size_t v = units_[pos] & 0x7FFFFFFFu;
        if (v >= outputs_.size()) return false;
        size_t e = outputs_.find('\0', v);
        out->assign(outputs_, v, (e == std::string::npos ? outputs_.size() : e) - v);
        return true;
      }
    }
    return false;
  }

  std::string normalize(const std::string& s) const {
    std::string out, rep;
    out.reserve(s.size());
    size_t i = 0;
    while (i < s.size()) {
      // grapheme [i, g)
      size_t g = i + utf8_len(static_cast<unsigned char>(s[i]));
      if (g > s.size()) g = s.size();
      const uint32_t base = decode_cp(s, i, int(g - i));
      const bool control = base < 0x20 || (base >= 0x7F && base <= 0x9F);  // never extended (UAX #29 GB4/GB5)
      if (s[i] == '\r' && g < s.size() && s[g] == '\n') ++g;
      while (!control && g < s.size()) {
        int n = utf8_len(static_cast<unsigned char>(s[g]));
        if (g + n > s.size() || !is_extender(decode_cp(s, g, n))) break;
        g += n;
      }
      if (g - i < 6 && transform(s.data() + i, g - i, &rep)) {
        out += rep;
      } else {
        for (size_t c = i; c < g;) {
          int n = utf8_len(static_cast<unsigned char>(s[c]));
          if (c + n > g) n = int(g - c);
          if (transform(s.data() + c, n, &rep)) out += rep;
          else out.append(s, c, n);
          c += n;
        }
      }
      i = g;
    }
    return out;
  }

 private:
  static bool has_leaf(uint32_t u) { return (u >> 8) & 1; }
  static uint32_t label(uint32_t u) { return u & ((1u << 31) | 0xFFu); }
  static uint32_t offset(uint32_t u) { return (u >> 10) << ((u & (1u << 9)) >> 6); }
  std::vector<uint32_t> units_;
  std::string outputs_;
};

// ---------------------------------------------------------------------------------------------
// Normalizer / pre-tokenizer steps
// ---------------------------------------------------------------------------------------------
struct NormStep {
  enum Kind { kCharsmap, kStrip, kReplace, kLowerAscii } kind;
  Charsmap map;
  bool left = false, right = false;
  bool regex = false;
  std::string pattern, content;
  std::regex re;
  // "<c>{n,}" / "<c>+" (T5's " {2,}"): collapsed by a direct scan instead of std::regex
  char run_char = 0;
  size_t run_min = 0;
};

inline std::string collapse_runs(const std::string& s, char c, size_t min_run, const std::string& with) {
  std::string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size();) {
    if (s[i] != c) { out.push_back(s[i++]); continue; }
    size_t j = i;
    while (j < s.size() && s[j] == c) ++j;
    if (j - i >= min_run) out += with;
    else out.append(s, i, j - i);
    i = j;
  }
  return out;
}

inline std::string strip_ws(const std::string& s, bool left, bool right) {
  size_t b = 0, e = s.size();
  if (left) {
    while (b < e) {
      int n = utf8_len(static_cast<unsigned char>(s[b]));
      if (b + n > e || !is_unicode_space(decode_cp(s, b, n))) break;
      b += n;
    }
  }
  if (right) {
    while (e > b) {
      size_t p = e - 1;
      while (p > b && (static_cast<unsigned char>(s[p]) & 0xC0) == 0x80) --p;
      if (!is_unicode_space(decode_cp(s, p, int(e - p)))) break;
      e = p;
    }
  }
  return s.substr(b, e - b);
}

inline std::string replace_all(const std::string& s, const std::string& pat, const std::string& with) {
  if (pat.empty()) return s;
  std::string out;
  size_t i = 0;
  for (size_t j; (j = s.find(pat, i)) != std::string::npos; i = j + pat.size()) out.append(s, i, j - i).append(with);
  return out.append(s, i, std::string::npos);
}

struct PreTok {
  bool whitespace_split = false;
  bool metaspace = false;
  std::string replacement = "\xE2\x96\x81";  // U+2581
  int prepend = 0;                           // 0 always, 1 first, 2 never
  bool split = true;
};

// ---------------------------------------------------------------------------------------------
// Unigram model
// ---------------------------------------------------------------------------------------------
class Unigram {
 public:
  Unigram() = default;
  Unigram(const std::vector<std::pair<std::string, double>>& vocab, int unk_id, bool fuse_unk)
      : unk_id_(unk_id), fuse_unk_(fuse_unk) {
    if (unk_id < 0 || unk_id >= int(vocab.size())) throw std::runtime_error("unigram: unk_id out of range");
    nodes_.emplace_back();
    double mn = 0.0;
    bool first = true;
    for (size_t id = 0; id < vocab.size(); ++id) {
      const std::string& p = vocab[id].first;
      ids_.emplace(p, int(id));
      if (first || vocab[id].second < mn) mn = vocab[id].second;
      first = false;
      if (p.empty()) continue;
      int cur = 0;
      for (unsigned char c : p) {
        int nxt = child(cur, c);
        if (nxt < 0) {
          nxt = int(nodes_.size());
          nodes_.emplace_back();
          nodes_[cur].kids.emplace_back(c, nxt);
        }
        cur = nxt;
      }
      if (nodes_[cur].id < 0) {  // first occurrence of a duplicated piece wins, as the id map
        nodes_[cur].id = int(id);
        nodes_[cur].score = vocab[id].second;
      }
    }
    unk_score_ = mn - 10.0;
    for (Node& nd : nodes_) std::sort(nd.kids.begin(), nd.kids.end());
    root_.fill(-1);
    for (auto& kv : nodes_[0].kids) root_[kv.first] = kv.second;
    dense_root_ = true;
  }

  // best segmentation of one pre-token into ids
  void encode(const std::string& s, std::vector<int>* out) const {
    const size_t n = s.size();
    if (!n) return;
    if (nodes_.empty()) throw std::runtime_error("unigram: no model loaded (call set_model first)");
    struct Best { double score = 0.0; long start = -1; int id = -1; };
    std::vector<Best> best(n + 1);
    best[0].start = 0;
    size_t at = 0;
    while (at < n) {
      const double base = best[at].score;
      const size_t mb = std::min<size_t>(utf8_len(static_cast<unsigned char>(s[at])), n - at);
      bool single = false;
      int cur = 0;
      for (size_t k = at; k < n; ++k) {
        cur = child(cur, static_cast<unsigned char>(s[k]));
        if (cur < 0) break;
        const Node& nd = nodes_[cur];
        if (nd.id < 0) continue;
        const size_t end = k + 1;
        const double cand = base + nd.score;
        if (best[end].start < 0 || cand > best[end].score) best[end] = {cand, long(at), nd.id};
        if (end - at == mb) single = true;
      }
      if (!single) {
        const double cand = base + unk_score_;
        Best& b = best[at + mb];
        if (b.start < 0 || cand > b.score) b = {cand, long(at), unk_id_};
      }
      at += mb;
    }
    // backtrack; runs of unknown pieces fuse into one token (looked up as a whole, else unk)
    std::vector<std::pair<size_t, size_t>> spans;  // reversed order
    std::vector<int> span_ids;
    size_t end = n;
    size_t unk_end = 0;
    bool in_unk = false;
    while (end > 0) {
      const Best& b = best[end];
      const size_t st = size_t(b.start);
      if (fuse_unk_ && b.id == unk_id_) {
        if (!in_unk) { unk_end = end; in_unk = true; }
      } else {
        if (in_unk) { spans.emplace_back(end, unk_end); span_ids.push_back(-1); in_unk = false; }
        spans.emplace_back(st, end);
        span_ids.push_back(b.id);
      }
      end = st;
    }
    if (in_unk) { spans.emplace_back(0, unk_end); span_ids.push_back(-1); }
    for (size_t i = spans.size(); i-- > 0;) {
      int id = span_ids[i];
      if (id < 0) {
        auto it = ids_.find(s.substr(spans[i].first, spans[i].second - spans[i].first));
        id = it == ids_.end() ? unk_id_ : it->second;
      }
      out->push_back(id);
    }
  }

 private:
  struct Node {
    std::vector<std::pair<unsigned char, int>> kids;
    int id = -1;
    double score = 0.0;
  };
  int child(int cur, unsigned char c) const {
    if (cur == 0 && dense_root_) return root_[c];
    const auto& k = nodes_[cur].kids;
    if (!dense_root_ || k.size() <= 8) {  // linear while building (edges unsorted) and for small fan-outs
      for (auto& kv : k)
        if (kv.first == c) return kv.second;
      return -1;
    }
    auto it = std::lower_bound(k.begin(), k.end(), std::make_pair(c, -1));
    return (it != k.end() && it->first == c) ? it->second : -1;
  }
  std::array<int, 256> root_{};
  bool dense_root_ = false;
  std::vector<Node> nodes_;
  std::unordered_map<std::string, int> ids_;
  int unk_id_ = 0;
  bool fuse_unk_ = true;
  double unk_score_ = -10.0;
};

// ---------------------------------------------------------------------------------------------
// Whole pipeline
// ---------------------------------------------------------------------------------------------
class Pipeline {
 public:
  std::vector<NormStep> norm;
  PreTok pre;
  Unigram model;
  std::vector<std::pair<std::string, int>> added;  // longest first
  std::array<std::vector<int>, 256> added_by_first;  // indices into `added` by first byte, longest first

  void set_added(std::vector<std::pair<std::string, int>> tokens) {
    std::stable_sort(tokens.begin(), tokens.end(),
                     [](const auto& a, const auto& b) { return a.first.size() > b.first.size(); });
    added = std::move(tokens);
    for (auto& v : added_by_first) v.clear();
    for (size_t a = 0; a < added.size(); ++a)
      if (!added[a].first.empty()) added_by_first[static_cast<unsigned char>(added[a].first[0])].push_back(int(a));
  }
  std::vector<int> suffix;                         // template post-processor: ids appended to a single sequence

  void add_charsmap(const std::string& blob) { NormStep s{NormStep::kCharsmap}; s.map = Charsmap(blob); norm.push_back(std::move(s)); }
  void add_strip(bool l, bool r) { NormStep s{NormStep::kStrip}; s.left = l; s.right = r; norm.push_back(std::move(s)); }
  void add_lower_ascii() { norm.push_back(NormStep{NormStep::kLowerAscii}); }
  void add_replace(const std::string& pattern, const std::string& content, bool regex) {
    NormStep s{NormStep::kReplace};
    s.pattern = pattern;
    s.content = content;
    s.regex = regex;
    if (regex) {
      static const std::regex run_form(R"(^([^\\\[\](){}.*+?^$|])(\{([0-9]+),\}|\+)$)");
      std::smatch m;
      if (std::regex_match(pattern, m, run_form)) {
        s.run_char = m[1].str()[0];
        s.run_min = m[3].matched ? std::stoul(m[3].str()) : 1;
      } else {
        s.re = std::regex(pattern, std::regex::ECMAScript | std::regex::optimize);
      }
    }
    norm.push_back(std::move(s));
  }

  std::string normalize(std::string s) const {
    for (const NormStep& st : norm) {
      switch (st.kind) {
        case NormStep::kCharsmap: s = st.map.normalize(s); break;
        case NormStep::kStrip: s = strip_ws(s, st.left, st.right); break;
        case NormStep::kLowerAscii:
          for (char& c : s) if (c >= 'A' && c <= 'Z') c = char(c - 'A' + 'a');
          break;
        case NormStep::kReplace:
          if (st.run_min) s = collapse_runs(s, st.run_char, st.run_min, st.content);
          else s = st.regex ? std::regex_replace(s, st.re, st.content) : replace_all(s, st.pattern, st.content);
          break;
      }
    }
    return s;
  }

  // normalized segment -> pre-tokens
  void pretokenize(const std::string& s, bool at_start, std::vector<std::string>* out) const {
    std::vector<std::pair<std::string, size_t>> words;  // (word, byte offset in s)
    if (pre.whitespace_split) {
      size_t i = 0, w = std::string::npos;
      while (i < s.size()) {
        int n = std::min<int>(utf8_len(static_cast<unsigned char>(s[i])), int(s.size() - i));
        if (is_unicode_space(decode_cp(s, i, n))) {
          if (w != std::string::npos) { words.emplace_back(s.substr(w, i - w), w); w = std::string::npos; }
        } else if (w == std::string::npos) {
          w = i;
        }
        i += n;
      }
      if (w != std::string::npos) words.emplace_back(s.substr(w), w);
    } else if (!s.empty()) {
      words.emplace_back(s, 0);
    }
    for (size_t wi = 0; wi < words.size(); ++wi) {
      std::string w = std::move(words[wi].first);
      if (!pre.metaspace) { out->push_back(std::move(w)); continue; }
      w = replace_all(w, " ", pre.replacement);
      const bool starts = w.compare(0, pre.replacement.size(), pre.replacement) == 0;
      // "first" prepends only to a piece that starts the original input
      if (!starts && (pre.prepend == 0 || (pre.prepend == 1 && at_start && words[wi].second == 0))) w = pre.replacement + w;
      if (!pre.split) { out->push_back(std::move(w)); continue; }
      // split on the replacement, each delimiter merged with the text after it
      size_t b = 0;
      for (size_t j = pre.replacement.size() <= w.size() ? w.find(pre.replacement, 1) : std::string::npos; j != std::string::npos;
           j = w.find(pre.replacement, j + 1)) {
        if (j > b) out->push_back(w.substr(b, j - b));
        b = j;
      }
      if (b < w.size()) out->push_back(w.substr(b));
    }
  }

  std::vector<int> encode(const std::string& text, bool add_special, long max_length, bool truncation) const {
    std::vector<int> ids;
    std::vector<std::string> pieces;
    size_t i = 0, seg = 0;
    auto flush = [&](size_t end) {
      if (end > seg) {
        pieces.clear();
        pretokenize(normalize(text.substr(seg, end - seg)), seg == 0, &pieces);
        for (const std::string& p : pieces) model.encode(p, &ids);
      }
    };
    while (i < text.size()) {
      int hit = -1;
      for (int a : added_by_first[static_cast<unsigned char>(text[i])]) {
        const std::string& t = added[a].first;
        if (text.compare(i, t.size(), t) == 0) { hit = a; break; }
      }
      if (hit >= 0) {
        flush(i);
        ids.push_back(added[hit].second);
        i += added[hit].first.size();
        seg = i;
      } else {
        i += std::max(1, utf8_len(static_cast<unsigned char>(text[i])));
      }
    }
    flush(text.size());
    const size_t extra = add_special ? suffix.size() : 0;
    if (truncation && max_length >= 0) {
      const size_t keep = size_t(max_length) > extra ? size_t(max_length) - extra : 0;
      if (ids.size() > keep) ids.resize(keep);
    }
    if (add_special) ids.insert(ids.end(), suffix.begin(), suffix.end());
    return ids;
  }
};

}  // namespace dalle_tok
