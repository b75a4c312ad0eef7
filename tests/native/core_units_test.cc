// core_units_test.cc -- CPU unit checks of the adapter core's containers
// (click_integration/elements/hip/hipcore.hh): the held-packet ring (a
// power-of-two ring with a kept mask, grown by doubling while it holds
// packets that wrapped) against a std::deque model, and a result chunk's
// put / at round trip.  No GPU, no glue library: run by tests/test_core_units.py.
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <random>
#include "../../click_integration/elements/hip/hipcore.hh"

namespace {
struct P {
    int id;
};
int fails = 0;
void check(bool ok, const char *what, long at)
{
    if (!ok && fails++ < 10)
        std::printf("FAIL %s at %ld\n", what, at);
}
}   // namespace

int main()
{
    // the ring: pushes and pops in bursts (a state holding two batches while
    // the older is routed), sizes crossing every power of two up to 2^15
    std::vector<P> pk(1 << 16);
    for (size_t k = 0; k < pk.size(); k++)
        pk[k].id = (int)k;
    hipcore::HeldRing<hipcore::Held<P> > ring;
    std::deque<hipcore::Held<P> > model;
    std::mt19937 rng(5);
    long next = 0, steps = 0;
    for (int round = 0; round < 400; round++) {
        const int push = (int)(rng() % 3000) + (round < 40 ? round * 400 : 0);
        for (int k = 0; k < push; k++, steps++) {
            hipcore::Held<P> e = {&pk[(size_t)(next % (long)pk.size())], nullptr, (uint32_t)next};
            next++;
            ring.push_back(e);
            model.push_back(e);
            check(ring.size() == model.size(), "size after push", steps);
        }
        if (!model.empty()) {                        // a pushed packet refused: pop_back
            ring.pop_back();
            model.pop_back();
        }
        const size_t pop = model.empty() ? 0 : rng() % (model.size() + 1);
        for (size_t k = 0; k < pop; k++, steps++) {
            check(ring.front().anno == model.front().anno && ring.front().p == model.front().p, "front", steps);
            ring.pop_front();
            model.pop_front();
        }
        for (size_t k = 0; k < model.size(); k += 1 + model.size() / 64)
            check(ring[k].anno == model[k].anno && ring[k].p == model[k].p, "index", (long)k);
        check(ring.size() == model.size() && ring.empty() == model.empty(), "size", round);
    }
    while (!model.empty()) {
        check(ring.front().anno == model.front().anno, "drain", (long)model.size());
        ring.pop_front();
        model.pop_front();
    }
    check(ring.empty(), "empty at the end", 0);
    std::printf("%s ring: %ld steps\n", fails ? "FAIL" : "PASS", steps);

    // a chunk entry: put then at gives the same result back
    const int before = fails;
    hipcore::Chunk<P> c;
    for (uint32_t k = 0; k < hipcore::Chunk<P>::CAP; k++) {
        hipcore::Routed<P> r = {&pk[k], k & 1 ? &pk[k + 1] : nullptr, k & 2 ? &pk[k + 2] : nullptr,
                                k & 4 ? &pk[k + 3] : nullptr, k * 3u, (int32_t)(k % 6) - 1, 1000 + k, k * 7u,
                                (int)(k % 5), (k & 8) != 0};
        c.put(k, r);
    }
    for (uint32_t k = 0; k < hipcore::Chunk<P>::CAP; k++) {
        const hipcore::Routed<P> r = c.at(k);
        check(r.p == &pk[k] && r.extra == (k & 1 ? &pk[k + 1] : nullptr) && r.made == (k & 2 ? &pk[k + 2] : nullptr) &&
                  r.parent == (k & 4 ? &pk[k + 3] : nullptr) && r.anno == k * 3u && r.port == (int32_t)(k % 6) - 1 &&
                  r.len == 1000 + k && r.aux == k * 7u && r.member == (int)(k % 5) && r.pass == ((k & 8) != 0),
              "chunk", k);
    }
    std::printf("%s chunk\n", fails > before ? "FAIL" : "PASS");
    std::printf("%s\n", fails ? "FAILED" : "ALL OK");
    return fails ? 1 : 0;
}
