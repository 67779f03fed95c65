// oaz_weights_io.cpp — model loading through the C ABI (the reference's only model entry is
// `vs.load(model_path)` in AlphaZeroMcts::from_model_file, alphazero-training/src/alphazero_mcts/
// mod.rs:89-105, on the ConvResNet built by net.rs:101-213).
//
//  * the canonical tensor table: the VarStore names net.rs creates, in creation order, with their
//    element counts (tch joins path components with '.' in memory and writes '|' into .ot files;
//    both spellings are accepted);
//  * named loading: a host hands over its variables as (name, data, numel) triples in any order
//    (e.g. tch's `vs.variables()` HashMap) and they are placed by name, every missing, duplicate,
//    unknown or wrongly sized tensor failing the load (Q13: the reference keeps its random weights
//    when the file does not match; here the load is refused with a message instead);
//  * an .ot reader: VarStore::save writes a TorchScript zip archive (stored members: data.pkl, one
//    data/<key> member per storage). data.pkl is interpreted opcode by opcode by a restricted
//    pickle machine that builds plain values only — nothing is imported, called or executed — and
//    only the `_rebuild_tensor_v2(storage, offset, shape, stride, ...)` records under the module's
//    state dict are used; tensor bytes come from the stored members (little-endian fp32).
// Host code only: no GPU is needed except to hand the result to an engine.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <map>
#include <string>
#include <vector>

#include "../../include/onitama_az.h"
#include "oaz_host.h"

namespace {

struct TensorSpec {
    std::string name;  // '|'-joined, as in the .ot files
    size_t numel;
    std::vector<size_t> shape;  // the tch shape (net.rs) the .ot writer records
};

// net.rs:101-213, in VarStore creation order (= oaz_weight_count's blob layout).
std::vector<TensorSpec> canonical_layout(int blocks) {
    std::vector<TensorSpec> v;
    const size_t C = 64, I = 21;
    auto add = [&](const std::string& n, std::vector<size_t> shape) {
        size_t numel = 1;
        for (size_t d : shape) numel *= d;
        v.push_back({n, numel, std::move(shape)});
    };
    auto conv = [&](const std::string& n, size_t cout, size_t cin, size_t k) {
        add(n + "|weight", {cout, cin, k, k});
        add(n + "|bias", {cout});
    };
    auto bn = [&](const std::string& n, size_t c) {
        for (const char* f : {"weight", "bias", "running_mean", "running_var"}) add(n + "|" + f, {c});
    };
    conv("conv_init_1", C, I, 3);
    bn("bn1", C);
    for (int i = 0; i < blocks; ++i)
        for (int j = 1; j <= 2; ++j) {
            const std::string p = "resnet_" + std::to_string(i) + "|resnet_small_block" + std::to_string(j);
            conv(p + "|small_block_conv", C, C, 3);
            bn(p + "|small_block_bn", C);
        }
    conv("vh_conv", 1, C, 1);
    bn("vh_bn", 1);
    add("vh_linear1|weight", {C, 25});
    add("vh_linear1|bias", {C});
    add("vh_linear2|weight", {1, C});
    add("vh_linear2|bias", {1});
    conv("policy_conv", 2, C, 1);
    bn("policy_bn", 2);
    add("ph_linear2|weight", {50, 50});
    add("ph_linear2|bias", {50});
    return v;
}

std::string normalise(const char* n) {
    std::string s(n);
    for (char& c : s)
        if (c == '.') c = '|';
    return s;
}

// Residual blocks of a name set: 1 + the largest i of "resnet_<i>|...", 0 without any.
int blocks_of(const std::vector<std::string>& names, int* out) {
    int mx = -1;
    for (const auto& n : names) {
        if (n.compare(0, 7, "resnet_") != 0) continue;
        char* end = nullptr;
        const long i = strtol(n.c_str() + 7, &end, 10);
        if (end == n.c_str() + 7 || *end != '|' || i < 0 || i > 63)
            return oaz_set_err(OAZ_ERR_WEIGHTS, "weights: unexpected tensor name '%s'", n.c_str());
        if (i > mx) mx = (int)i;
    }
    *out = mx + 1;
    return 0;
}

int assemble(int blocks, const std::vector<std::string>& names, const std::vector<const float*>& data,
             const std::vector<size_t>& sizes, float* out, size_t cap) {
    const auto layout = canonical_layout(blocks);
    const size_t need = oaz_weight_count(blocks, 64, 21);
    if (!out || cap < need) return oaz_set_err(OAZ_ERR_ARG, "weights: output holds %zu floats, need %zu", cap, need);
    std::map<std::string, size_t> at;
    for (size_t i = 0; i < names.size(); ++i)
        if (!at.emplace(names[i], i).second)
            return oaz_set_err(OAZ_ERR_WEIGHTS, "weights: tensor '%s' given twice", names[i].c_str());
    size_t off = 0, used = 0;
    for (const auto& t : layout) {
        auto it = at.find(t.name);
        if (it == at.end())  // VarStore::load: TensorNameNotFound
            return oaz_set_err(OAZ_ERR_WEIGHTS, "weights: missing tensor '%s' (%d-block ResNet, net.rs:101-213)",
                               t.name.c_str(), blocks);
        const size_t i = it->second;
        if (sizes[i] != t.numel)
            return oaz_set_err(OAZ_ERR_WEIGHTS, "weights: tensor '%s' has %zu elements, expected %zu", t.name.c_str(),
                               sizes[i], t.numel);
        if (!data[i]) return oaz_set_err(OAZ_ERR_ARG, "weights: tensor '%s' has no data", t.name.c_str());
        memcpy(out + off, data[i], t.numel * sizeof(float));
        off += t.numel;
        ++used;
    }
    if (used != names.size())
        for (const auto& n : names) {
            bool known = false;
            for (const auto& t : layout) known = known || t.name == n;
            if (!known)
                return oaz_set_err(OAZ_ERR_WEIGHTS, "weights: tensor '%s' is not part of a %d-block ResNet", n.c_str(),
                                   blocks);
        }
    if (off != need) return oaz_set_err(OAZ_ERR_STATE, "weights: layout mismatch");
    return 0;
}

// ---- zip (stored members) ---------------------------------------------------------------------
uint32_t rd16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
uint32_t rd32(const uint8_t* p) { return rd16(p) | (rd16(p + 2) << 16); }
uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

struct Member {
    uint64_t data_off, size;
    uint32_t method;
};

int zip_index(const std::vector<uint8_t>& f, std::map<std::string, Member>& out) {
    const size_t n = f.size();
    if (n < 22) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: not a zip archive");
    size_t eocd = SIZE_MAX;
    for (size_t i = n - 22 + 1; i-- > 0 && n - i <= 22 + 65535;)
        if (rd32(&f[i]) == 0x06054b50u) {
            eocd = i;
            break;
        }
    if (eocd == SIZE_MAX) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: no zip end-of-central-directory record");
    uint64_t entries = rd16(&f[eocd + 10]), cd_off = rd32(&f[eocd + 16]);
    if ((entries == 0xFFFF || cd_off == 0xFFFFFFFFu) && eocd >= 20 && rd32(&f[eocd - 20]) == 0x07064b50u) {
        const uint64_t z64 = rd64(&f[eocd - 20 + 8]);  // zip64 end-of-central-directory record
        if (z64 > n || n - z64 < 56 || rd32(&f[z64]) != 0x06064b50u)
            return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: bad zip64 record");
        entries = rd64(&f[z64 + 32]);
        cd_off = rd64(&f[z64 + 48]);
    }
    uint64_t p = cd_off;
    for (uint64_t k = 0; k < entries; ++k) {
        // (every bound is checked by subtraction: offsets and sizes come from the file and may be near 2^64)
        if (p > n || n - p < 46 || rd32(&f[p]) != 0x02014b50u)
            return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: bad central directory");
        const uint32_t method = rd16(&f[p + 10]);
        uint64_t size = rd32(&f[p + 24]), local = rd32(&f[p + 42]);
        const uint32_t nl = rd16(&f[p + 28]), xl = rd16(&f[p + 30]), cl = rd16(&f[p + 32]);
        if (n - p - 46 < (uint64_t)nl + xl + cl) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: truncated central directory");
        std::string name((const char*)&f[p + 46], nl);
        const uint64_t xend = p + 46 + nl + xl;
        for (uint64_t x = p + 46 + nl; x + 4 <= xend;) {  // zip64 extra: sizes / offset
            const uint32_t id = rd16(&f[x]), len = rd16(&f[x + 2]);
            if (x + 4 + len > xend) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: bad zip extra field");
            if (id == 0x0001) {
                uint64_t q = x + 4;
                if (size == 0xFFFFFFFFu && q + 8 <= x + 4 + len) size = rd64(&f[q]), q += 8;  // uncompressed
                if (rd32(&f[p + 20]) == 0xFFFFFFFFu && q + 8 <= x + 4 + len) q += 8;           // compressed
                if (local == 0xFFFFFFFFu && q + 8 <= x + 4 + len) local = rd64(&f[q]);
            }
            x += 4 + len;
        }
        if (local > n || n - local < 30 || rd32(&f[local]) != 0x04034b50u)
            return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: bad local header");
        const uint64_t data = local + 30 + rd16(&f[local + 26]) + rd16(&f[local + 28]);
        if (method == 0 && (data > n || n - data < size))
            return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: member '%s' truncated", name.c_str());
        out[name] = Member{data, size, method};
        p += 46 + nl + xl + cl;
    }
    return 0;
}

// ---- restricted pickle machine ----------------------------------------------------------------
// Values live in one arena owned by the caller and refer to each other by index, so a crafted
// data.pkl cannot build what a pointer graph would make dangerous: memo aliasing (BINPUT / BINGET)
// may still create shared or cyclic containers, but releasing the arena is one flat free (no
// recursive destructor, no leaked cycle), and find_tensors visits every value at most once with
// an explicit stack (no exponential walk over aliased paths, no native-stack recursion). The arena,
// the stack, the container references and the marks are capped.
constexpr uint32_t kNil = 0xFFFFFFFFu;
constexpr size_t kMaxValues = 1u << 18;   // a VarStore data.pkl holds ~15 values per tensor
constexpr size_t kMaxRefs = 1u << 20;     // container items over the whole file
constexpr size_t kMaxStack = 1u << 16;    // stack entries + marks
struct Val {
    enum Kind : uint8_t { NONE, BOOL, INT, FLOAT, STR, TUPLE, LIST, DICT, GLOBAL, PERSID, CALL } k = NONE;
    int64_t i = 0;
    double f = 0;
    std::string s;                // STR; GLOBAL "module name"
    std::vector<uint32_t> items;  // TUPLE / LIST; DICT as key, value pairs
    uint32_t callee = kNil, args = kNil, state = kNil;  // CALL (REDUCE / NEWOBJ, BUILD state); PERSID args
};
using Arena = std::vector<Val>;

int unpickle(const uint8_t* p, size_t n, Arena& A, uint32_t* result) {
    std::vector<uint32_t> st;
    std::vector<size_t> marks;
    std::map<uint64_t, uint32_t> memo;
    size_t i = 0, refs = 0;
    auto need = [&](size_t k) { return k <= n - i; };
    auto bad = [&](const char* what) { return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: data.pkl: %s at byte %zu", what, i); };
    auto mk = [&](Val::Kind k, uint32_t* out) {
        if (A.size() >= kMaxValues || st.size() + marks.size() >= kMaxStack) return false;
        A.emplace_back();
        A.back().k = k;
        *out = (uint32_t)(A.size() - 1);
        return true;
    };
    auto push = [&](uint32_t v) {
        if (st.size() + marks.size() >= kMaxStack) return false;
        st.push_back(v);
        return true;
    };
    auto pop = [&](uint32_t* v) {
        if (st.empty()) return false;
        *v = st.back();
        st.pop_back();
        return true;
    };
    auto line = [&](std::string* s) {
        const uint8_t* e = (const uint8_t*)memchr(p + i, '\n', n - i);
        if (!e) return false;
        s->assign((const char*)p + i, (size_t)(e - (p + i)));
        i = (size_t)(e - p) + 1;
        return true;
    };
    auto push_str = [&](size_t len) {
        uint32_t v;
        if (!need(len) || !mk(Val::STR, &v)) return false;
        A[v].s.assign((const char*)p + i, len);
        i += len;
        st.push_back(v);
        return true;
    };
    auto push_int = [&](int64_t x) {
        uint32_t v;
        if (!mk(Val::INT, &v)) return false;
        A[v].i = x;
        st.push_back(v);
        return true;
    };
    auto since_mark = [&](std::vector<uint32_t>* out) {
        if (marks.empty() || marks.back() > st.size()) return false;
        out->assign(st.begin() + (long)marks.back(), st.end());
        st.resize(marks.back());
        marks.pop_back();
        return true;
    };
    // Adds items to container c (a LIST or DICT; anything else ignores them, as the Python walker
    // does). A container may not hold itself: that is the one cycle a VarStore pickle never has and
    // a crafted one needs.
    auto extend = [&](uint32_t c, const uint32_t* xs, size_t k) {
        for (size_t j = 0; j < k; ++j)
            if (xs[j] == c) return false;
        if (k > kMaxRefs - refs) return false;
        refs += k;
        A[c].items.insert(A[c].items.end(), xs, xs + k);
        return true;
    };
    while (i < n) {
        const uint8_t op = p[i++];
        uint32_t a, b, c;
        std::vector<uint32_t> xs;
        switch (op) {
            case 0x80: if (!need(1)) return bad("PROTO"); i += 1; break;   // PROTO
            case 0x95: if (!need(8)) return bad("FRAME"); i += 8; break;   // FRAME
            case '.':                                                      // STOP
                if (st.empty()) return bad("empty stack at STOP");
                *result = st.back();
                return 0;
            case 'X': if (!need(4) || !(i += 4, push_str(rd32(p + i - 4)))) return bad("BINUNICODE"); break;
            case 0x8c: if (!need(1) || !(i += 1, push_str(p[i - 1]))) return bad("SHORT_BINUNICODE"); break;
            case 'U': if (!need(1) || !(i += 1, push_str(p[i - 1]))) return bad("SHORT_BINSTRING"); break;
            case 'T': if (!need(4) || !(i += 4, push_str(rd32(p + i - 4)))) return bad("BINSTRING"); break;
            case 'K': if (!need(1) || !push_int(p[i])) return bad("BININT1"); i += 1; break;
            case 'M': if (!need(2) || !push_int(rd16(p + i))) return bad("BININT2"); i += 2; break;
            case 'J': if (!need(4) || !push_int((int32_t)rd32(p + i))) return bad("BININT"); i += 4; break;
            case 0x8a: {  // LONG1: little-endian two's complement of n bytes
                if (!need(1) || p[i] > 8 || !need(1 + (size_t)p[i])) return bad("LONG1");
                const int len = p[i++];
                uint64_t u = 0;
                for (int k = 0; k < len; ++k) u |= (uint64_t)p[i + k] << (8 * k);
                if (len > 0 && len < 8 && (p[i + len - 1] & 0x80)) u |= ~0ull << (8 * len);
                i += (size_t)len;
                if (!push_int((int64_t)u)) return bad("LONG1");
                break;
            }
            case 'G': {  // BINFLOAT: big-endian double
                if (!need(8) || !mk(Val::FLOAT, &a)) return bad("BINFLOAT");
                uint64_t u = 0;
                for (int k = 0; k < 8; ++k) u = (u << 8) | p[i + k];
                i += 8;
                memcpy(&A[a].f, &u, 8);
                st.push_back(a);
                break;
            }
            case 0x88: if (!mk(Val::BOOL, &a)) return bad("NEWTRUE"); A[a].i = 1; st.push_back(a); break;
            case 0x89: if (!mk(Val::BOOL, &a)) return bad("NEWFALSE"); st.push_back(a); break;
            case 'N': if (!mk(Val::NONE, &a)) return bad("NONE"); st.push_back(a); break;
            case 'c': {  // GLOBAL: recorded as a name, never resolved
                std::string m, nm;
                if (!line(&m) || !line(&nm) || !mk(Val::GLOBAL, &a)) return bad("GLOBAL");
                A[a].s = m + " " + nm;
                st.push_back(a);
                break;
            }
            case 'q': if (!need(1) || st.empty()) return bad("BINPUT"); memo[p[i]] = st.back(); i += 1; break;
            case 'r': if (!need(4) || st.empty()) return bad("LONG_BINPUT"); memo[rd32(p + i)] = st.back(); i += 4; break;
            case 0x94:
                if (st.empty() || memo.size() >= kMaxValues) return bad("MEMOIZE");
                memo[memo.size()] = st.back();
                break;
            case 'h':
                if (!need(1) || !memo.count(p[i]) || !push(memo[p[i]])) return bad("BINGET");
                i += 1;
                break;
            case 'j':
                if (!need(4) || !memo.count(rd32(p + i)) || !push(memo[rd32(p + i)])) return bad("LONG_BINGET");
                i += 4;
                break;
            case '(':
                if (st.size() + marks.size() >= kMaxStack) return bad("MARK");
                marks.push_back(st.size());
                break;
            case 't':
                if (!since_mark(&xs) || !mk(Val::TUPLE, &a) || xs.size() > kMaxRefs - refs) return bad("TUPLE");
                refs += xs.size();
                A[a].items = xs;
                st.push_back(a);
                break;
            case ')': if (!mk(Val::TUPLE, &a)) return bad("EMPTY_TUPLE"); st.push_back(a); break;
            case 0x85: case 0x86: case 0x87: {  // TUPLE1..3
                const size_t k = op - 0x84u;
                if (st.size() < k) return bad("TUPLEn");
                xs.assign(st.end() - (long)k, st.end());
                st.resize(st.size() - k);
                if (k > kMaxRefs - refs || !mk(Val::TUPLE, &a)) return bad("TUPLEn");
                A[a].items = xs;
                refs += k;
                st.push_back(a);
                break;
            }
            case '}': if (!mk(Val::DICT, &a)) return bad("EMPTY_DICT"); st.push_back(a); break;
            case ']': if (!mk(Val::LIST, &a)) return bad("EMPTY_LIST"); st.push_back(a); break;
            case 'u':  // SETITEMS
                if (!since_mark(&xs) || st.empty() || (xs.size() & 1)) return bad("SETITEMS");
                if (A[st.back()].k == Val::DICT && !extend(st.back(), xs.data(), xs.size())) return bad("SETITEMS");
                break;
            case 's':  // SETITEM
                if (!pop(&b) || !pop(&a) || st.empty()) return bad("SETITEM");
                xs = {a, b};
                if (A[st.back()].k == Val::DICT && !extend(st.back(), xs.data(), 2)) return bad("SETITEM");
                break;
            case 'e':  // APPENDS
                if (!since_mark(&xs) || st.empty()) return bad("APPENDS");
                if (A[st.back()].k == Val::LIST && !extend(st.back(), xs.data(), xs.size())) return bad("APPENDS");
                break;
            case 'a':  // APPEND
                if (!pop(&a) || st.empty()) return bad("APPEND");
                if (A[st.back()].k == Val::LIST && !extend(st.back(), &a, 1)) return bad("APPEND");
                break;
            case 'Q':  // BINPERSID
                if (!pop(&a) || !mk(Val::PERSID, &b)) return bad("BINPERSID");
                A[b].args = a;
                st.push_back(b);
                break;
            case 'R': case 0x81:  // REDUCE / NEWOBJ: recorded as a call, never made
                if (!pop(&b) || !pop(&a) || !mk(Val::CALL, &c)) return bad("REDUCE");
                A[c].callee = a;
                A[c].args = b;
                st.push_back(c);
                break;
            case 'b':  // BUILD
                if (!pop(&a) || st.empty()) return bad("BUILD");
                if (A[st.back()].k == Val::CALL) A[st.back()].state = a;
                break;
            default: {
                char msg[48];
                snprintf(msg, sizeof(msg), "unsupported opcode 0x%02x", op);
                return bad(msg);
            }
        }
    }
    return bad("no STOP");
}

struct TensorRec {
    std::string key;
    int64_t offset;
    std::vector<int64_t> shape, stride;
};

// One `_rebuild_tensor_v2(persid, offset, shape, stride, requires_grad, hooks)` record -> TensorRec.
int tensor_record(const Arena& A, const std::string& name, uint32_t args, TensorRec* r) {
    auto is = [&](uint32_t v, Val::Kind k) { return v != kNil && A[v].k == k; };
    if (!is(args, Val::TUPLE) || A[args].items.size() < 4 || !is(A[args].items[0], Val::PERSID))
        return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: tensor '%s': unexpected record", name.c_str());
    const std::vector<uint32_t>& a = A[args].items;
    const uint32_t pers = A[a[0]].args;  // ('storage', <dtype storage>, key, location, numel)
    if (!is(pers, Val::TUPLE) || A[pers].items.size() < 3 || !is(A[pers].items[2], Val::STR))
        return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: tensor '%s': unexpected storage record", name.c_str());
    const uint32_t ty = A[pers].items[1];
    if (!is(ty, Val::GLOBAL) || A[ty].s != "torch FloatStorage")
        return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: tensor '%s': storage %s (fp32 only)", name.c_str(),
                           is(ty, Val::GLOBAL) ? A[ty].s.c_str() : "?");
    r->key = A[A[pers].items[2]].s;
    if (!is(a[1], Val::INT)) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: '%s': bad offset", name.c_str());
    r->offset = A[a[1]].i;
    for (int w = 2; w <= 3; ++w) {
        if (!is(a[w], Val::TUPLE) || A[a[w]].items.size() > 6)
            return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: '%s': bad shape", name.c_str());
        for (uint32_t d : A[a[w]].items) {
            if (!is(d, Val::INT)) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: '%s': bad shape", name.c_str());
            (w == 2 ? r->shape : r->stride).push_back(A[d].i);
        }
    }
    if (r->shape.size() != r->stride.size()) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: '%s': bad shape/stride", name.c_str());
    return 0;
}

bool is_rebuild(const Arena& A, uint32_t v) {
    return v != kNil && A[v].k == Val::CALL && A[v].callee != kNil && A[A[v].callee].k == Val::GLOBAL &&
           A[A[v].callee].s == "torch._utils _rebuild_tensor_v2";
}

// name -> _rebuild_tensor_v2 record, from every dict reachable from the root (the module's state).
// Depth-first over an explicit stack; every value is expanded once (shared and cyclic values too).
int find_tensors(const Arena& A, uint32_t root, std::map<std::string, TensorRec>& out) {
    std::vector<uint8_t> seen(A.size(), 0);
    std::vector<uint32_t> todo;
    if (root != kNil) todo.push_back(root);
    while (!todo.empty()) {
        const uint32_t v = todo.back();
        todo.pop_back();
        if (seen[v]) continue;
        seen[v] = 1;
        const Val& x = A[v];
        if (x.k == Val::DICT) {
            for (size_t j = 0; j + 1 < x.items.size(); j += 2) {
                const uint32_t key = x.items[j], val = x.items[j + 1];
                if (A[key].k == Val::STR && is_rebuild(A, val)) {
                    TensorRec r;
                    if (int rc = tensor_record(A, A[key].s, A[val].args, &r)) return rc;
                    out[A[key].s] = r;
                } else if (!seen[val]) {
                    todo.push_back(val);
                }
            }
        } else if (x.k == Val::TUPLE || x.k == Val::LIST) {
            for (uint32_t y : x.items)
                if (!seen[y]) todo.push_back(y);
        } else if (x.k == Val::CALL) {
            if (x.args != kNil && !seen[x.args]) todo.push_back(x.args);
            if (x.state != kNil && !seen[x.state]) todo.push_back(x.state);
        }
    }
    return 0;
}

int read_ot(const char* path, int* blocks_out, std::vector<float>* blob) {
    FILE* fp = fopen(path, "rb");
    if (!fp) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: cannot open '%s'", path);
    std::vector<uint8_t> f;
    fseek(fp, 0, SEEK_END);
    const long len = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    if (len > 0) {
        f.resize((size_t)len);
        if (fread(f.data(), 1, f.size(), fp) != f.size()) f.clear();
    }
    fclose(fp);
    if (f.empty()) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: cannot read '%s'", path);
    std::map<std::string, Member> zm;
    if (int rc = zip_index(f, zm)) return rc;
    std::string root;
    const Member* pkl = nullptr;
    for (const auto& kv : zm) {
        const std::string& n = kv.first;
        if (n == "data.pkl" || (n.size() > 9 && n.compare(n.size() - 9, 9, "/data.pkl") == 0 &&
                                n.find('/') == n.size() - 9)) {
            root = n.substr(0, n.size() - 8);
            pkl = &kv.second;
            break;
        }
    }
    if (!pkl) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: '%s' has no data.pkl", path);
    if (pkl->method != 0) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: data.pkl is compressed (stored members expected)");
    std::map<std::string, TensorRec> recs;
    {
        Arena arena;
        uint32_t top = kNil;
        if (int rc = unpickle(&f[pkl->data_off], (size_t)pkl->size, arena, &top)) return rc;
        if (int rc = find_tensors(arena, top, recs)) return rc;
    }
    std::vector<std::string> names;
    std::vector<std::vector<float>> vals;
    for (const auto& kv : recs) {
        const TensorRec& r = kv.second;
        auto it = zm.find(root + "data/" + r.key);
        if (it == zm.end() || it->second.method != 0)
            return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: tensor '%s': storage member data/%s missing or compressed",
                               kv.first.c_str(), r.key.c_str());
        const size_t avail = (size_t)(it->second.size / 4);
        const uint8_t* base = &f[it->second.data_off];
        size_t numel = 1;
        for (size_t d = 0; d < r.shape.size(); ++d) {
            const int64_t sz = r.shape[d], sd = r.stride[d];
            if (sz < 0 || sd < 0 || (uint64_t)sd > avail)
                return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: tensor '%s': bad size or stride", kv.first.c_str());
            if (sz > 0 && numel > avail / (size_t)sz)  // a parameter holds at most its storage's elements
                return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: tensor '%s' is larger than its storage", kv.first.c_str());
            numel *= (size_t)sz;
        }
        std::vector<float> out(numel);
        std::vector<int64_t> idx(r.shape.size(), 0);
        for (size_t e = 0; e < numel; ++e) {  // strided gather in row-major order
            int64_t src = r.offset;
            for (size_t d = 0; d < idx.size(); ++d) src += idx[d] * r.stride[d];
            if (src < 0 || (size_t)src >= avail)
                return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: tensor '%s' reaches past its storage", kv.first.c_str());
            uint32_t u = rd32(base + 4 * (size_t)src);
            memcpy(&out[e], &u, 4);
            for (size_t d = idx.size(); d-- > 0;) {
                if (++idx[d] < r.shape[d]) break;
                idx[d] = 0;
            }
        }
        names.push_back(normalise(kv.first.c_str()));
        vals.push_back(std::move(out));
    }
    int blocks = 0;
    if (int rc = blocks_of(names, &blocks)) return rc;
    std::vector<const float*> data;
    std::vector<size_t> sizes;
    for (const auto& v : vals) data.push_back(v.data()), sizes.push_back(v.size());
    blob->assign(oaz_weight_count(blocks, 64, 21), 0.0f);
    if (int rc = assemble(blocks, names, data, sizes, blob->data(), blob->size())) return rc;
    *blocks_out = blocks;
    return 0;
}

// ---- .ot writer (save_vs, alphazero-training/src/train.rs:414-430: `vs.save(&path)`) ------------
// The archive VarStore::save produces and VarStore::load / oaz_ot_read / torch.jit.load read: a zip
// of stored members under "<file stem>/": data/<i> (tensor i's little-endian fp32 bytes, data
// 64-byte aligned by an "FB" padding extra field, as torch's own writer aligns them), data.pkl (a
// protocol-2 pickle of a `__torch__.Module` whose state dict maps each '|' name to
// torch._utils._rebuild_tensor_v2(storage i, 0, shape, contiguous stride, False, OrderedDict())),
// code/__torch__.py (the module's parameter list), constants.pkl and version. Every member is
// stored (the reference's files deflate code/__torch__.py; no reader depends on that). The byte
// layout is the one weights.write_ot (Python zipfile) emits for the same tensors, which
// tests/test_host.py checks byte for byte.
struct Bytes {
    std::string b;
    void u8(uint32_t v) { b.push_back((char)(v & 0xFF)); }
    void u16(uint32_t v) { u8(v), u8(v >> 8); }
    void u32(uint32_t v) { u16(v & 0xFFFF), u16(v >> 16); }
    void raw(const void* p, size_t n) { b.append((const char*)p, n); }
    void str(const std::string& s) { b += s; }
};

struct Crc32Table {
    uint32_t t[256];
    constexpr Crc32Table() : t{} {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            t[i] = c;
        }
    }
};
constexpr Crc32Table kCrc32;  // built at compile time: no lazy initialisation shared between threads

uint32_t crc32(const uint8_t* p, size_t n) {
    const uint32_t* table = kCrc32.t;
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}

// pickle protocol-2 pieces (weights.py _pk_str / _pk_int / _pk_tuple)
void pk_str(Bytes& o, const std::string& s) {
    o.str("X");
    o.u32((uint32_t)s.size());
    o.str(s);
}
void pk_int(Bytes& o, size_t v) {
    if (v < 256) {
        o.str("K");
        o.u8((uint32_t)v);
    } else if (v < 65536) {
        o.str("M");
        o.u16((uint32_t)v);
    } else {
        o.str("J");
        o.u32((uint32_t)v);
    }
}

std::string data_pkl(const std::vector<TensorSpec>& layout) {
    Bytes o;
    o.str(std::string("\x80\x02", 2));
    o.str("c__torch__\nModule\n)\x81}(");
    for (size_t i = 0; i < layout.size(); ++i) {
        const TensorSpec& t = layout[i];
        pk_str(o, t.name);
        o.str("ctorch._utils\n_rebuild_tensor_v2\n(");
        o.str("(");  // persistent id: ('storage', FloatStorage, key, location, numel)
        pk_str(o, "storage");
        o.str("ctorch\nFloatStorage\n");
        pk_str(o, std::to_string(i));
        pk_str(o, "cpu");
        pk_int(o, t.numel);
        o.str("tQ");
        pk_int(o, 0);  // storage offset
        o.str("(");
        for (size_t d : t.shape) pk_int(o, d);
        o.str("t(");
        std::vector<size_t> stride(t.shape.size());
        size_t acc = 1;
        for (size_t d = t.shape.size(); d-- > 0;) stride[d] = acc, acc *= t.shape[d];
        for (size_t sd : stride) pk_int(o, sd);
        o.str("t\x89");  // requires_grad False
        o.str("ccollections\nOrderedDict\n)Rt");
        o.str("R");
    }
    o.str("ub.");
    return o.b;
}

std::string torch_py(const std::vector<TensorSpec>& layout) {
    std::string s = "class Module(Module):\n  __parameters__ = [";
    for (const auto& t : layout) s += "\"" + t.name + "\", ";
    s += "]\n  __buffers__ = []\n  __annotations__ = []\n";
    for (const auto& t : layout) s += "  __annotations__[\"" + t.name + "\"] = Tensor\n";
    return s;
}

struct ZipWriter {
    Bytes out, cd;
    uint32_t count = 0;
    void add(const std::string& name, const void* data, size_t n) {
        const uint32_t off = (uint32_t)out.b.size();
        const uint32_t crc = crc32((const uint8_t*)data, n);
        const size_t start = off + 30 + name.size();
        const uint32_t pad = (uint32_t)((64 - (start + 4) % 64) % 64);  // data starts 64-byte aligned
        std::string extra = "FB";
        extra.push_back((char)(pad & 0xFF));
        extra.push_back((char)(pad >> 8));
        extra.append(pad, 'Z');
        auto common = [&](Bytes& h) {  // flags, method (stored), DOS time 0:00:00, date 1980-01-01, crc, sizes
            h.u16(0), h.u16(0), h.u16(0), h.u16((0 << 9) | (1 << 5) | 1);
            h.u32(crc), h.u32((uint32_t)n), h.u32((uint32_t)n);
            h.u16((uint32_t)name.size()), h.u16((uint32_t)extra.size());
        };
        out.u32(0x04034b50u);
        out.u8(20), out.u8(0);  // version needed 2.0
        common(out);
        out.str(name);
        out.str(extra);
        out.raw(data, n);
        cd.u32(0x02014b50u);
        cd.u8(20), cd.u8(3), cd.u8(20), cd.u8(0);  // made by 2.0 on Unix, needs 2.0
        common(cd);
        cd.u16(0), cd.u16(0), cd.u16(0);  // comment length, disk, internal attributes
        cd.u32(0600u << 16);              // external attributes: a regular file, rw-------
        cd.u32(off);
        cd.str(name);
        cd.str(extra);
        ++count;
    }
    std::string finish() {
        const uint32_t cd_off = (uint32_t)out.b.size(), cd_size = (uint32_t)cd.b.size();
        out.str(cd.b);
        out.u32(0x06054b50u);
        out.u16(0), out.u16(0), out.u16(count), out.u16(count);
        out.u32(cd_size), out.u32(cd_off);
        out.u16(0);
        return out.b;
    }
};

int write_ot(const char* path, const float* blob, size_t n, int blocks) {
    const auto layout = canonical_layout(blocks);
    const size_t need = oaz_weight_count(blocks, 64, 21);
    if (n != need) return oaz_set_err(OAZ_ERR_ARG, "ot_write: %zu floats given, a %d-block network has %zu", n, blocks, need);
    std::string stem(path);
    const size_t slash = stem.find_last_of('/');
    if (slash != std::string::npos) stem = stem.substr(slash + 1);
    const size_t dot = stem.find_last_of('.');
    if (dot != std::string::npos && dot > 0) stem = stem.substr(0, dot);
    if (stem.empty()) return oaz_set_err(OAZ_ERR_ARG, "ot_write: bad path '%s'", path);
    ZipWriter z;
    size_t off = 0;
    std::vector<uint8_t> le;
    for (size_t i = 0; i < layout.size(); ++i) {
        le.resize(layout[i].numel * 4);
        for (size_t e = 0; e < layout[i].numel; ++e) {  // little-endian fp32
            uint32_t u;
            memcpy(&u, blob + off + e, 4);
            for (int k = 0; k < 4; ++k) le[4 * e + k] = (uint8_t)(u >> (8 * k));
        }
        off += layout[i].numel;
        z.add(stem + "/data/" + std::to_string(i), le.data(), le.size());
    }
    const std::string pkl = data_pkl(layout), code = torch_py(layout);
    z.add(stem + "/data.pkl", pkl.data(), pkl.size());
    z.add(stem + "/code/__torch__.py", code.data(), code.size());
    z.add(stem + "/constants.pkl", "\x80\x02).", 4);
    z.add(stem + "/version", "3\n", 2);
    const std::string bytes = z.finish();
    if (bytes.size() >= 0xFFFFFFFFull) return oaz_set_err(OAZ_ERR_ARG, "ot_write: archive too large");
    // written beside the target and renamed over it: a reader never sees a half-written checkpoint
    const std::string tmp = std::string(path) + ".tmp";
    FILE* fp = fopen(tmp.c_str(), "wb");
    if (!fp) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot_write: cannot create '%s'", tmp.c_str());
    const bool ok = fwrite(bytes.data(), 1, bytes.size(), fp) == bytes.size();
    if (fclose(fp) != 0 || !ok) {
        remove(tmp.c_str());
        return oaz_set_err(OAZ_ERR_WEIGHTS, "ot_write: cannot write '%s'", tmp.c_str());
    }
    if (rename(tmp.c_str(), path) != 0) {
        remove(tmp.c_str());
        return oaz_set_err(OAZ_ERR_WEIGHTS, "ot_write: cannot rename '%s' to '%s'", tmp.c_str(), path);
    }
    return 0;
}

}  // namespace

extern "C" size_t oaz_weight_tensor_count(int blocks) {
    return blocks < 0 ? 0 : canonical_layout(blocks).size();
}

extern "C" int oaz_weight_tensor_info(int blocks, size_t i, char* name, size_t name_cap, size_t* numel) {
    if (blocks < 0) return oaz_set_err(OAZ_ERR_ARG, "weight_tensor_info: blocks < 0");
    const auto layout = canonical_layout(blocks);
    if (i >= layout.size()) return oaz_set_err(OAZ_ERR_ARG, "weight_tensor_info: index %zu of %zu", i, layout.size());
    if (numel) *numel = layout[i].numel;
    if (name) {
        if (name_cap <= layout[i].name.size()) return oaz_set_err(OAZ_ERR_ARG, "weight_tensor_info: name buffer too small");
        memcpy(name, layout[i].name.c_str(), layout[i].name.size() + 1);
    }
    return 0;
}

extern "C" int oaz_weights_from_named(int blocks, const char* const* names, const float* const* data,
                                      const size_t* sizes, size_t n, float* out, size_t out_n) {
    if (blocks < 0 || (n && (!names || !data || !sizes))) return oaz_set_err(OAZ_ERR_ARG, "weights_from_named: bad arguments");
    std::vector<std::string> nm;
    for (size_t i = 0; i < n; ++i) {
        if (!names[i]) return oaz_set_err(OAZ_ERR_ARG, "weights_from_named: name %zu is null", i);
        nm.push_back(normalise(names[i]));
    }
    return assemble(blocks, nm, std::vector<const float*>(data, data + n), std::vector<size_t>(sizes, sizes + n), out,
                    out_n);
}

extern "C" int oaz_load_weights_named(oaz_engine* e, const char* const* names, const float* const* data,
                                      const size_t* sizes, size_t n) {
    oaz_config cfg;
    if (int rc = oaz_get_config(e, &cfg)) return rc;
    std::vector<float> blob(oaz_weight_count(cfg.blocks, 64, 21));
    if (int rc = oaz_weights_from_named(cfg.blocks, names, data, sizes, n, blob.data(), blob.size())) return rc;
    return oaz_load_weights(e, blob.data(), blob.size());
}

extern "C" int oaz_ot_read(const char* path, float* out, size_t cap, size_t* n_out, int* blocks_out) {
    if (!path) return oaz_set_err(OAZ_ERR_ARG, "ot_read: null path");
    std::vector<float> blob;
    int blocks = 0;
    if (int rc = read_ot(path, &blocks, &blob)) return rc;
    if (n_out) *n_out = blob.size();
    if (blocks_out) *blocks_out = blocks;
    if (out) {
        if (cap < blob.size()) return oaz_set_err(OAZ_ERR_CAPACITY, "ot_read: %zu floats needed, cap %zu", blob.size(), cap);
        memcpy(out, blob.data(), blob.size() * sizeof(float));
    }
    return 0;
}

extern "C" int oaz_load_ot(oaz_engine* e, const char* path) {
    oaz_config cfg;
    if (int rc = oaz_get_config(e, &cfg)) return rc;
    std::vector<float> blob;
    int blocks = 0;
    if (int rc = read_ot(path, &blocks, &blob)) return rc;
    if (blocks != cfg.blocks)
        return oaz_set_err(OAZ_ERR_WEIGHTS, "load_ot: '%s' holds a %d-block ResNet, the engine was made for %d", path,
                           blocks, cfg.blocks);
    return oaz_load_weights(e, blob.data(), blob.size());
}

extern "C" int oaz_ot_write(const char* path, const float* blob, size_t n, int blocks) {
    if (!path || !blob || blocks < 0 || blocks > 64) return oaz_set_err(OAZ_ERR_ARG, "ot_write: bad arguments");
    return write_ot(path, blob, n, blocks);
}

extern "C" int oaz_checkpoint_path(const char* folder, int64_t iteration, int is_best, const char* stamp, char* out,
                                   size_t cap) {
    if (!folder || !out || iteration < 0) return oaz_set_err(OAZ_ERR_ARG, "checkpoint_path: bad arguments");
    char now[32];
    if (!stamp) {  // Local::now().format("%Y%m%d_%H%M%S")
        const time_t t = time(nullptr);
        struct tm tm;
        localtime_r(&t, &tm);
        strftime(now, sizeof now, "%Y%m%d_%H%M%S", &tm);
        stamp = now;
    }
    const int len = snprintf(out, cap, "%s/%smodel_%lld_%s.ot", folder, is_best ? "best_" : "", (long long)iteration, stamp);
    if (len < 0 || (size_t)len >= cap) return oaz_set_err(OAZ_ERR_CAPACITY, "checkpoint_path: %d bytes needed", len + 1);
    return 0;
}
