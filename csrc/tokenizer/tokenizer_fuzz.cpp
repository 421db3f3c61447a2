// Sanitizer driver for the native caption tokenizer: the pybind-free core
// (unigram_core.h) is built with ThreadSanitizer or AddressSanitizer + UBSan by
// tests/test_tokenizer_cpu.py and fed random byte strings -- ASCII, valid multi-byte UTF-8, truncated
// and invalid sequences, special tokens, whitespace runs -- from several threads sharing one Pipeline
// (the batch encoder's sharing pattern). Captions are untrusted input; every id must stay in range.
//
//   tokenizer_fuzz <spec dir: vocab.tsv [charsmap.bin]> <threads> <strings per thread>
#include <atomic>
#include <cstdio>
#include <fstream>
#include <random>
#include <sstream>
#include <thread>

#include "unigram_core.h"

using dalle_tok::Pipeline;

static std::string random_text(std::mt19937& rng) {
  static const char* pieces[] = {"a", "red", " ", "  ", "\t", "\n", "</s>", "<pad>", "caf\xC3\xA9", "\xEF\xAC\x81",
                                 "\xE2\x91\xA0", "\xEF\xBC\xA6", "\xE4\xB8\xAD", "\xF0\x9F\x98\x80", "\xE2\x80\x8D",
                                 "\xCC\x81", "\r\n", "\xE3\x80\x80", "!!", "2021"};
  std::string s;
  const int n = rng() % 48;
  for (int i = 0; i < n; ++i) {
    const unsigned r = rng() % 10;
    if (r < 6) {
      s += pieces[rng() % (sizeof(pieces) / sizeof(pieces[0]))];
    } else if (r < 8) {
      s.push_back(char(32 + rng() % 95));
    } else {
      s.push_back(char(rng() % 256));  // arbitrary byte: lone continuation bytes, truncated leads, NUL
    }
  }
  if (rng() % 4 == 0 && !s.empty()) s.pop_back();  // often cut inside a multi-byte sequence
  return s;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <spec dir> <threads> <strings per thread>\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int threads = std::atoi(argv[2]), per = std::atoi(argv[3]);
  std::vector<std::pair<std::string, double>> vocab;
  {
    std::ifstream f(dir + "/vocab.tsv", std::ios::binary);
    std::string line;
    while (std::getline(f, line)) {
      const size_t tab = line.rfind('\t');
      if (tab == std::string::npos) continue;
      vocab.emplace_back(line.substr(0, tab), std::stod(line.substr(tab + 1)));
    }
  }
  if (vocab.size() < 4) {
    std::fprintf(stderr, "vocab.tsv: too few pieces\n");
    return 2;
  }
  Pipeline p;
  {
    std::ifstream f(dir + "/charsmap.bin", std::ios::binary);
    if (f) {
      std::stringstream ss;
      ss << f.rdbuf();
      p.add_charsmap(ss.str());
    }
  }
  p.add_strip(false, true);
  p.add_replace(" {2,}", "\xE2\x96\x81", true);
  p.add_replace("x+", "x", true);  // exercises the std::regex fallback too (not a run of one char)
  p.add_replace("ab", "b", false);
  p.pre.whitespace_split = true;
  p.pre.metaspace = true;
  p.model = dalle_tok::Unigram(vocab, 2, true);
  p.set_added({{"<pad>", 0}, {"</s>", 1}});
  p.suffix = {1};
  std::atomic<long> tokens{0}, bad{0};
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      std::mt19937 rng(1234 + t);
      for (int i = 0; i < per; ++i) {
        const std::string s = random_text(rng);
        const auto ids = p.encode(s, i & 1, (i % 3) ? -1 : long(rng() % 12), (i % 3) == 0);
        for (int id : ids)
          if (id < 0 || id >= int(vocab.size())) bad.fetch_add(1);
        tokens.fetch_add(long(ids.size()));
        (void)p.normalize(s);
      }
    });
  for (auto& th : pool) th.join();
  if (bad.load()) {
    std::fprintf(stderr, "%ld ids out of range\n", bad.load());
    return 1;
  }
  std::printf("tokenizer fuzz ok: %d threads x %d strings, %ld tokens\n", threads, per, tokens.load());
  return 0;
}
