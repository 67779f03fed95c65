// cpu_baseline.cpp — TEST/MEASUREMENT INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
//
// The reference-equivalent CPU baseline of BASELINE.md §4 / SURVEY.md 8d: the reference's
// self-play execution shape with its NN on libtorch's CPU kernels, because the Rust/tch binary
// cannot be built here (no rustc/cargo, no LibTorch 1.13.1):
//   - one game per worker thread, workers = the host's physical cores, each worker's searches
//     sequential (alphazero-training/src/train.rs:218-245: thread_amnt workers, private models);
//   - one batch-1 NN forward per simulation (mcts_arena.rs:156, 267-273 -> net.rs:215-232),
//     through ATen CPU ops (conv2d, batch_norm eval, relu, linear, tanh, softmax: the ops tch
//     calls; torch 2.10's ATen stands in for libtorch 1.13.1), intra-op threads 1 per worker;
//   - the MCTS itself is the C oracle's restatement of mcts_arena.rs (oracle/oaz_oracle.c),
//     fed through its evaluator callback.
// Output: one JSON object on stdout.
//
//   oaz_cpu_baseline bench <weights.f32> <blocks> <sims> <threads> <seconds> <fixed_deck 0|1>
//   oaz_cpu_baseline c1    <weights.f32> <blocks> <sims>           (one whole game, one thread)
//   oaz_cpu_baseline nn    <weights.f32> <blocks> <states.bin> <out.f32>  (batch-1 forwards of n
//                          oaz_state records -> n x (50 policy + 1 value) floats; tests/ pin the
//                          evaluator against the torch goldens with it)
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <c10/core/InferenceMode.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "oaz_oracle.h"

namespace {

// The canonical blob (tch VarStore order, include/onitama_az.h oaz_weight_count) as named tensors.
struct Net {
    int blocks = 0;
    std::map<std::string, at::Tensor> t;
};

void take(Net& n, const float*& p, const std::string& name, std::vector<int64_t> shape) {
    int64_t k = 1;
    for (auto s : shape) k *= s;
    n.t[name] = at::from_blob(const_cast<float*>(p), shape, at::kFloat).clone();
    p += k;
}

void take_conv_bn(Net& n, const float*& p, const std::string& conv, const std::string& bn, int64_t cout, int64_t cin,
                  int64_t k) {
    take(n, p, conv + ".weight", {cout, cin, k, k});
    take(n, p, conv + ".bias", {cout});
    take(n, p, bn + ".weight", {cout});
    take(n, p, bn + ".bias", {cout});
    take(n, p, bn + ".running_mean", {cout});
    take(n, p, bn + ".running_var", {cout});
}

Net load_net(const std::vector<float>& blob, int blocks) {
    Net n;
    n.blocks = blocks;
    const float* p = blob.data();
    take_conv_bn(n, p, "conv_init_1", "bn1", 64, 21, 3);
    for (int i = 0; i < blocks; ++i)
        for (int j = 1; j <= 2; ++j) {
            const std::string b = "resnet_" + std::to_string(i) + ".resnet_small_block" + std::to_string(j);
            take_conv_bn(n, p, b + ".small_block_conv", b + ".small_block_bn", 64, 64, 3);
        }
    take_conv_bn(n, p, "vh_conv", "vh_bn", 1, 64, 1);
    take(n, p, "vh_linear1.weight", {64, 25});
    take(n, p, "vh_linear1.bias", {64});
    take(n, p, "vh_linear2.weight", {1, 64});
    take(n, p, "vh_linear2.bias", {1});
    take_conv_bn(n, p, "policy_conv", "policy_bn", 2, 64, 1);
    take(n, p, "ph_linear2.weight", {50, 50});
    take(n, p, "ph_linear2.bias", {50});
    if ((size_t)(p - blob.data()) != blob.size()) {
        fprintf(stderr, "weights: %zu floats consumed of %zu\n", (size_t)(p - blob.data()), blob.size());
        exit(2);
    }
    return n;
}

at::Tensor cbn(const Net& n, const at::Tensor& x, const std::string& conv, const std::string& bn, int64_t pad) {
    const auto& t = n.t;
    at::Tensor y = at::conv2d(x, t.at(conv + ".weight"), t.at(conv + ".bias"), {1, 1}, {pad, pad});
    return at::batch_norm(y, t.at(bn + ".weight"), t.at(bn + ".bias"), t.at(bn + ".running_mean"),
                          t.at(bn + ".running_var"), false, 0.1, 1e-5, false);
}

// ConvResNet::forward(xs, train=false), net.rs:215-232 (ResTower net.rs:101-212)
void forward(const Net& n, const at::Tensor& x, float* policy, float* value) {
    c10::InferenceMode guard;
    at::Tensor y = at::relu(cbn(n, x, "conv_init_1", "bn1", 1));
    for (int i = 0; i < n.blocks; ++i) {
        const std::string b = "resnet_" + std::to_string(i) + ".resnet_small_block";
        at::Tensor h = at::relu(cbn(n, y, b + "1.small_block_conv", b + "1.small_block_bn", 1));
        h = cbn(n, h, b + "2.small_block_conv", b + "2.small_block_bn", 1);
        y = at::relu(h + y);
    }
    at::Tensor v = at::relu(cbn(n, y, "vh_conv", "vh_bn", 0)).flatten(1);
    v = at::relu(at::linear(v, n.t.at("vh_linear1.weight"), n.t.at("vh_linear1.bias")));
    v = at::tanh(at::linear(v, n.t.at("vh_linear2.weight"), n.t.at("vh_linear2.bias")));
    at::Tensor pp = at::relu(cbn(n, y, "policy_conv", "policy_bn", 0)).flatten(1);
    pp = at::softmax(at::linear(pp, n.t.at("ph_linear2.weight"), n.t.at("ph_linear2.bias")), -1);
    pp = pp.contiguous();
    memcpy(policy, pp.data_ptr<float>(), 50 * sizeof(float));
    *value = v.item<float>();
}

// evaluate (mcts_arena.rs:267-273): create_tensor_from_state (common.rs:26-80) -> [1,21,5,5] -> forward
void eval_cb(void* ctx, const oaz_state* s, float policy[50], float* value) {
    const Net& n = *static_cast<const Net*>(ctx);
    float planes[21 * 25];
    orc_encode(s, s->to_move, planes);
    at::Tensor x = at::from_blob(planes, {1, 21, 5, 5}, at::kFloat);
    forward(n, x, policy, value);
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

orc_selfplay_cfg make_cfg(const Net* net, int sims, int fixed_deck) {
    orc_selfplay_cfg c;
    memset(&c, 0, sizeof(c));
    c.search.sims = sims;
    c.search.c_puct = 5.0;      // bin/train.rs:54
    c.search.train_noise = 1;   // bin/train.rs:55
    c.search.alpha = 0.03;
    c.search.eps = 0.25;
    c.search.seed = 20260101ull;
    c.search.evaluator = 2;     // callback
    c.search.fn = eval_cb;
    c.search.ctx = const_cast<Net*>(net);
    c.max_plies = 150;
    c.fixed_deck = fixed_deck;
    for (int i = 0; i < 5; ++i) c.deck[i] = (uint8_t)i;  // [Tiger, Dragon, Frog, Rabbit, Crab]
    return c;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 5 || (std::string(argv[1]) == "nn" && argc < 6)) {
        fprintf(stderr, "usage: %s bench|c1|nn weights.f32 blocks sims|states [threads seconds fixed_deck]|out\n",
                argv[0]);
        return 2;
    }
    const std::string mode = argv[1];
    const int blocks = atoi(argv[3]), sims = mode == "nn" ? 0 : atoi(argv[4]);
    FILE* f = fopen(argv[2], "rb");
    if (!f) {
        fprintf(stderr, "cannot open %s\n", argv[2]);
        return 2;
    }
    std::vector<float> blob(orc_weight_count(blocks));
    if (fread(blob.data(), sizeof(float), blob.size(), f) != blob.size()) {
        fprintf(stderr, "short weights file\n");
        return 2;
    }
    fclose(f);
    at::set_num_threads(1);  // one intra-op thread: each worker thread runs its own batch-1 forwards
    const Net net = load_net(blob, blocks);
    if (mode == "nn") {
        FILE* fs = fopen(argv[4], "rb");
        FILE* fo = fopen(argv[5], "wb");
        if (!fs || !fo) return 2;
        oaz_state s;
        while (fread(&s, sizeof(s), 1, fs) == 1) {
            float out[51];
            eval_cb(const_cast<Net*>(&net), &s, out, &out[50]);
            fwrite(out, sizeof(float), 51, fo);
        }
        fclose(fs);
        fclose(fo);
        return 0;
    }
    if (mode == "c1") {  // BASELINE C1: one game, fixed deck, one thread
        orc_selfplay_cfg c = make_cfg(&net, sims, 1);
        std::vector<oaz_sample> out(160);
        int result = 0, plies = 0;
        oaz_search_stats st;
        memset(&st, 0, sizeof(st));
        const double t0 = now_s();
        const int n = orc_selfplay_game(&c, 0, out.data(), (int)out.size(), &result, &plies, &st);
        const double dt = now_s() - t0;
        if (n < 0) return 1;
        printf("{\"mode\": \"c1\", \"seconds\": %.6f, \"sims\": %llu, \"plies\": %d, \"games\": 1, \"result\": %d, "
               "\"sims_per_s\": %.3f, \"games_per_s\": %.6f, \"threads\": 1}\n",
               dt, (unsigned long long)st.sims, plies, result, (double)st.sims / dt, 1.0 / dt);
        return 0;
    }
    if (argc < 8) return 2;
    const int threads = atoi(argv[5]), fixed = atoi(argv[7]);
    const double seconds = atof(argv[6]);
    orc_selfplay_cfg c = make_cfg(&net, sims, fixed);
    int64_t games = 0, plies = 0;
    const double t0 = now_s();
    const int64_t done = orc_selfplay_bench(&c, threads, seconds, &games, &plies);
    const double dt = now_s() - t0;
    printf("{\"mode\": \"bench\", \"seconds\": %.6f, \"sims\": %lld, \"plies\": %lld, \"games\": %lld, "
           "\"sims_per_s\": %.3f, \"games_per_s\": %.6f, \"threads\": %d}\n",
           dt, (long long)done, (long long)plies, (long long)games, (double)done / dt, (double)games / dt, threads);
    return 0;
}
