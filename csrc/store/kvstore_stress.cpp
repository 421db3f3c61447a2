// Multi-threaded stress driver for the native key/value store (kvstore_core.h), built by
// tests/test_kvstore_sanitizers_cpu.py with -fsanitize=thread and with -fsanitize=address,undefined
// (host code only; SURVEY §5.2 race detection). Exit status 0 and no sanitizer report = pass.
//
// Phases (each asserts its own invariants):
//   1. contention: T threads, each with its own client, hammer overlapping keys with STORE / GET /
//      KEYS / DELETE while owner-tagged subkeys must never be overwritten by another owner;
//   2. barrier: N clients rendezvous through server-side WAIT (the matchmaking primitive);
//   3. churn: clients connect, issue a request and disconnect repeatedly (worker reaping path);
//   4. shutdown: stop() while clients are parked in WAIT with a long timeout must return promptly,
//      and a client whose server went away must fail with an exception, not hang or crash.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "kvstore_core.h"

using namespace dalle_kv;

#define CHECK(cond)                                                                 \
  do {                                                                              \
    if (!(cond)) {                                                                  \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      std::exit(2);                                                                 \
    }                                                                               \
  } while (0)

static double secs_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
  const int threads = argc > 1 ? std::atoi(argv[1]) : 8;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 300;
  KVServer server("127.0.0.1", 0);
  const int port = server.port();

  // 1. contention on shared keys; every peer owns its subkey (pre-registered, so a forged write by
  //    another peer always meets a live owned record and must be refused)
  {
    const double base = now_s() + 1000.0;
    {
      ClientCore c("127.0.0.1", port, 5.0);
      for (int k = 0; k < 7; ++k)
        for (int t = 0; t < threads; ++t) {
          const std::string me = "peer" + std::to_string(t);
          CHECK(c.store("k" + std::to_string(k), me, "init", base, me));
        }
    }
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) {
      ts.emplace_back([&, t] {
        ClientCore c("127.0.0.1", port, 5.0);
        const std::string me = "peer" + std::to_string(t);
        const std::string other = "peer" + std::to_string((t + 1) % threads);
        for (int i = 0; i < iters; ++i) {
          const std::string key = "k" + std::to_string(i % 7);
          const double exp = base + 1.0 + i;  // strictly later than this peer's previous write
          CHECK(c.store(key, me, me + ":" + std::to_string(i), exp, me));
          CHECK(!c.store(key, me, "stale", exp - 0.5, me));                       // older value refused
          if (threads > 1) CHECK(!c.store(key, other, "forged", exp + 1e4, me));  // not my subkey
          auto v = c.get(key);
          CHECK(v.size() == (size_t)threads);
          for (auto& e : v) CHECK(std::get<1>(e) != "forged" && std::get<1>(e) != "stale");
          if (i % 50 == 0) c.keys("k");
          if (i % 97 == 0) c.store("tmp" + me, "x", "y", now_s() + 0.001, "");  // expires almost at once
          if (i % 101 == 0) c.del("tmp" + me);
        }
      });
    }
    for (auto& t : ts) t.join();
  }

  // 2. barrier through server-side WAIT
  {
    const int n = threads;
    std::vector<std::thread> ts;
    std::atomic<int> released{0};
    for (int t = 0; t < n; ++t) {
      ts.emplace_back([&, t] {
        ClientCore c("127.0.0.1", port, 5.0);
        CHECK(c.store("barrier", "p" + std::to_string(t), "1", now_s() + 60.0, ""));
        uint32_t live = c.wait("barrier", (uint32_t)n, 20.0);
        CHECK(live >= (uint32_t)n);
        released++;
      });
    }
    for (auto& t : ts) t.join();
    CHECK(released.load() == n);
  }

  // 3. connection churn (server reaps finished workers while accepting new ones)
  {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) {
      ts.emplace_back([&] {
        for (int i = 0; i < iters / 10 + 1; ++i) {
          ClientCore c("127.0.0.1", port, 5.0);
          CHECK(c.ping());
        }
      });
    }
    for (auto& t : ts) t.join();
  }

  // 4. stop() with clients parked in a long WAIT
  {
    std::vector<std::thread> ts;
    std::atomic<int> returned{0};
    std::atomic<int> ready{0};
    for (int t = 0; t < threads; ++t) {
      ts.emplace_back([&] {
        ClientCore c("127.0.0.1", port, 5.0);
        ready++;
        try {
          c.wait("never", 1000, 120.0);  // far longer than the test may take
        } catch (const std::exception&) {
        }
        returned++;
      });
    }
    while (ready.load() < threads) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    std::this_thread::sleep_for(std::chrono::milliseconds(200));  // let the WAITs reach the server
    const auto t0 = std::chrono::steady_clock::now();
    server.stop();
    for (auto& t : ts) t.join();
    const double dt = secs_since(t0);
    CHECK(returned.load() == threads);
    CHECK(dt < 10.0);
    std::printf("stop() with %d parked waiters: %.3f s\n", threads, dt);
  }

  // a client of a dead server fails loudly
  {
    bool threw = false;
    try {
      ClientCore c("127.0.0.1", port, 0.2);
      c.ping();
    } catch (const std::exception&) {
      threw = true;
    }
    CHECK(threw);
  }
  std::printf("kvstore stress ok: %d threads x %d iters\n", threads, iters);
  return 0;
}
