// Host-side index stream of the reference's MultiPassRandomSampler
// (utils/samplers.py:25-34): per epoch the generator is re-seeded with
// base_seed + epoch, keys = torch.rand((num_passes, data_len)) and the order is the
// UNSTABLE argsort of each row, flattened.  Reproducing the stream bit for bit needs
// torch's CPU MT19937 (a strictly sequential generator) and torch's CPU sort, which is
// libstdc++ introsort over (key, index) pairs; ~500 keys per 131072-key pass tie, and
// the tie order is fixed only by introsort's partition history.  Neither piece has a
// parallel formulation with the same output, so this stays on the host: MT19937 draws
// run once, the passes are sorted on worker threads, and the runtime uploads the
// int32 stream once per rollout (overlapped with the device update of the previous
// epoch by the Python host, see gsamd/samplers.py).
#include <stdint.h>

#include <algorithm>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/gsamd.h"

namespace gs {
void set_error(const char *fmt, ...);
}

namespace {

class TorchMT19937 {
  public:
    explicit TorchMT19937(uint64_t seed)
    {
        state_[0] = (uint32_t)(seed & 0xffffffffu);
        for (int i = 1; i < kN; ++i) state_[i] = 1812433253u * (state_[i - 1] ^ (state_[i - 1] >> 30)) + (uint32_t)i;
        pos_ = kN;
    }
    uint32_t operator()()
    {
        if (pos_ == kN) twist();
        uint32_t y = state_[pos_++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        return y ^ (y >> 18);
    }

  private:
    static constexpr int kN = 624, kM = 397;
    void twist()
    {
        for (int i = 0; i < kN; ++i) {
            const uint32_t y = (state_[i] & 0x80000000u) | (state_[(i + 1) % kN] & 0x7fffffffu);
            state_[i] = state_[(i + kM) % kN] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        pos_ = 0;
    }
    uint32_t state_[kN];
    int pos_;
};

void sort_pass(const float *keys, int64_t n, int32_t *out)
{
    std::vector<std::pair<float, int64_t>> kv((size_t)n);
    for (int64_t i = 0; i < n; ++i) kv[(size_t)i] = {keys[i], i};
    std::sort(kv.begin(), kv.end(),
              [](const std::pair<float, int64_t> &a, const std::pair<float, int64_t> &b) { return a.first < b.first; });
    for (int64_t i = 0; i < n; ++i) out[i] = (int32_t)kv[(size_t)i].second;
}

}  // namespace

extern "C" int gs_sampler_stream_i32(int64_t data_len, int64_t num_passes, uint64_t seed, int32_t *out, int n_threads)
{
    if (data_len <= 0 || num_passes <= 0 || data_len > INT32_MAX || !out) {
        gs::set_error("gs_sampler_stream_i32: data_len and num_passes must be > 0 (got %lld, %lld)",
                      (long long)data_len, (long long)num_passes);
        return GS_E_INVALID;
    }
    // torch.rand(float32): 24 low bits of each 32-bit draw times 2^-24, row-major
    std::vector<float> keys((size_t)(data_len * num_passes));
    TorchMT19937 gen(seed);
    for (auto &k : keys) k = (float)(gen() & 0xFFFFFFu) * (1.0f / 16777216.0f);
    int nt = n_threads < 1 ? 1 : n_threads;
    if (nt > num_passes) nt = (int)num_passes;
    if (nt == 1) {
        for (int64_t p = 0; p < num_passes; ++p) sort_pass(keys.data() + p * data_len, data_len, out + p * data_len);
        return GS_OK;
    }
    std::vector<std::thread> pool;
    for (int w = 0; w < nt; ++w) {
        pool.emplace_back([&, w]() {
            for (int64_t p = w; p < num_passes; p += nt) sort_pass(keys.data() + p * data_len, data_len, out + p * data_len);
        });
    }
    for (auto &t : pool) t.join();
    return GS_OK;
}
