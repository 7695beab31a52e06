// Actor runtime tests (mirrors the reference's master/pkg/actor/*_test.go behaviours).
#include <atomic>
#include <string>

#include "detcore/actor.h"
#include "test_util.h"

using namespace detcore::actor;

namespace {
struct Add {
  int v;
};
struct Get {};
struct Boom {};

class Counter : public Actor {
 public:
  explicit Counter(std::atomic<int>* poststops) : poststops_(poststops) {}
  void Receive(Context& ctx) override {
    if (auto a = ctx.As<Add>()) total_ += a->v;
    else if (ctx.Is<Get>()) ctx.Respond(total_);
    else if (ctx.Is<Boom>()) throw std::runtime_error("boom");
    else if (ctx.Is<PostStop>()) ++*poststops_;
  }

 private:
  int total_ = 0;
  std::atomic<int>* poststops_;
};
}  // namespace

TEST(actor_tell_ask_ordering) {
  System sys(4);
  std::atomic<int> ps{0};
  Ref c = sys.ActorOf("counter", std::make_unique<Counter>(&ps));
  for (int i = 1; i <= 1000; ++i) c->Tell(Add{i});
  Message m = c->AskSync(Get{});
  EXPECT(m.has_value());
  EXPECT_EQ(std::any_cast<int>(m), 500500);
  EXPECT(sys.Get("/counter") == c);
  c->Stop();
  EXPECT(c->AwaitTermination(std::chrono::milliseconds(5000)));
  EXPECT_EQ(ps.load(), 1);
  EXPECT(!c->AskSync(Get{}, std::chrono::milliseconds(100)).has_value());  // stopped: no response
  sys.Shutdown();
}

TEST(actor_no_response_is_empty) {
  System sys(2);
  std::atomic<int> ps{0};
  Ref c = sys.ActorOf("c", std::make_unique<Counter>(&ps));
  Message m = c->AskSync(Add{1});
  EXPECT(!m.has_value());
  sys.Shutdown();
  EXPECT_EQ(ps.load(), 1);
}

TEST(actor_children_stop_first_and_failure_reaches_parent) {
  System sys(3);
  std::atomic<int> ps{0};
  std::atomic<int> child_failed{0}, child_stopped{0};
  Ref parent = sys.ActorOf("parent", std::make_unique<FuncActor>([&](Context& ctx) {
    if (ctx.Is<PreStart>()) {
      ctx.ActorOf("a", std::make_unique<Counter>(&ps));
      ctx.ActorOf("b", std::make_unique<Counter>(&ps));
    } else if (auto s = ctx.As<std::string>()) {
      if (*s == "boom") ctx.Tell(ctx.Child("a"), Boom{});
      if (*s == "count") ctx.Respond(static_cast<int>(ctx.Children().size()));
    } else if (ctx.Is<ChildFailed>()) {
      ++child_failed;
    } else if (ctx.Is<ChildStopped>()) {
      ++child_stopped;
    }
  }));
  EXPECT_EQ(std::any_cast<int>(parent->AskSync(std::string("count"))), 2);
  EXPECT(sys.Get("/parent/a") != nullptr);
  parent->Tell(std::string("boom"));
  for (int i = 0; i < 200 && child_failed.load() == 0; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(5));
  EXPECT_EQ(child_failed.load(), 1);
  EXPECT_EQ(std::any_cast<int>(parent->AskSync(std::string("count"))), 1);
  parent->Stop();
  EXPECT(parent->AwaitTermination(std::chrono::milliseconds(5000)));
  EXPECT_EQ(ps.load(), 2);  // both children ran PostStop (failed one included)
  EXPECT_EQ(child_stopped.load(), 1);
  sys.Shutdown();
}

TEST(actor_notify_after) {
  System sys(2);
  std::atomic<int> got{0};
  Ref r = sys.ActorOf("t", std::make_unique<FuncActor>([&](Context& ctx) {
    if (ctx.Is<int>()) got = *ctx.As<int>();
  }));
  auto t0 = std::chrono::steady_clock::now();
  sys.NotifyAfter(r, std::chrono::milliseconds(50), 7);
  while (got.load() == 0 && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2))
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  EXPECT_EQ(got.load(), 7);
  EXPECT(std::chrono::steady_clock::now() - t0 >= std::chrono::milliseconds(45));
  sys.Shutdown();
}
