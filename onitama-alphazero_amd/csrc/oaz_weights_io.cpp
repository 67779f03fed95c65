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

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/onitama_az.h"
#include "oaz_host.h"

namespace {

struct TensorSpec {
    std::string name;  // '|'-joined, as in the .ot files
    size_t numel;
};

// net.rs:101-213, in VarStore creation order (= oaz_weight_count's blob layout).
std::vector<TensorSpec> canonical_layout(int blocks) {
    std::vector<TensorSpec> v;
    const size_t C = 64, I = 21;
    auto conv = [&](const std::string& n, size_t cout, size_t cin, size_t k) {
        v.push_back({n + "|weight", cout * cin * k * k});
        v.push_back({n + "|bias", cout});
    };
    auto bn = [&](const std::string& n, size_t c) {
        for (const char* f : {"weight", "bias", "running_mean", "running_var"}) v.push_back({n + "|" + f, c});
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
    v.push_back({"vh_linear1|weight", C * 25});
    v.push_back({"vh_linear1|bias", C});
    v.push_back({"vh_linear2|weight", C});
    v.push_back({"vh_linear2|bias", 1});
    conv("policy_conv", 2, C, 1);
    bn("policy_bn", 2);
    v.push_back({"ph_linear2|weight", 2500});
    v.push_back({"ph_linear2|bias", 50});
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
struct Val;
using V = std::shared_ptr<Val>;
struct Val {
    enum Kind { NONE, BOOL, INT, FLOAT, STR, TUPLE, LIST, DICT, GLOBAL, PERSID, CALL } k = NONE;
    int64_t i = 0;
    double f = 0;
    std::string s;             // STR; GLOBAL "module name"
    std::vector<V> items;      // TUPLE / LIST; DICT as key, value pairs
    V callee, args, state;     // CALL (REDUCE / NEWOBJ, BUILD state); PERSID args
};
V mk(Val::Kind k) {
    auto v = std::make_shared<Val>();
    v->k = k;
    return v;
}

int unpickle(const uint8_t* p, size_t n, V* result) {
    std::vector<V> st;
    std::vector<size_t> marks;
    std::map<uint64_t, V> memo;
    size_t i = 0;
    auto need = [&](size_t k) { return i + k <= n; };
    auto bad = [&](const char* what) { return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: data.pkl: %s at byte %zu", what, i); };
    auto pop = [&](V* v) {
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
        if (!need(len)) return false;
        V v = mk(Val::STR);
        v->s.assign((const char*)p + i, len);
        i += len;
        st.push_back(v);
        return true;
    };
    auto since_mark = [&](std::vector<V>* out) {
        if (marks.empty() || marks.back() > st.size()) return false;
        out->assign(st.begin() + (long)marks.back(), st.end());
        st.resize(marks.back());
        marks.pop_back();
        return true;
    };
    while (i < n) {
        const uint8_t op = p[i++];
        V a, b, c;
        std::vector<V> xs;
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
            case 'K': if (!need(1)) return bad("BININT1"); a = mk(Val::INT); a->i = p[i]; i += 1; st.push_back(a); break;
            case 'M': if (!need(2)) return bad("BININT2"); a = mk(Val::INT); a->i = rd16(p + i); i += 2; st.push_back(a); break;
            case 'J': if (!need(4)) return bad("BININT"); a = mk(Val::INT); a->i = (int32_t)rd32(p + i); i += 4; st.push_back(a); break;
            case 0x8a: {  // LONG1: little-endian two's complement of n bytes
                if (!need(1) || !need(1 + (size_t)p[i]) || p[i] > 8) return bad("LONG1");
                const int len = p[i++];
                uint64_t u = 0;
                for (int k = 0; k < len; ++k) u |= (uint64_t)p[i + k] << (8 * k);
                if (len > 0 && len < 8 && (p[i + len - 1] & 0x80)) u |= ~0ull << (8 * len);
                i += (size_t)len;
                a = mk(Val::INT);
                a->i = (int64_t)u;
                st.push_back(a);
                break;
            }
            case 'G': {  // BINFLOAT: big-endian double
                if (!need(8)) return bad("BINFLOAT");
                uint64_t u = 0;
                for (int k = 0; k < 8; ++k) u = (u << 8) | p[i + k];
                i += 8;
                a = mk(Val::FLOAT);
                memcpy(&a->f, &u, 8);
                st.push_back(a);
                break;
            }
            case 0x88: a = mk(Val::BOOL); a->i = 1; st.push_back(a); break;  // NEWTRUE
            case 0x89: a = mk(Val::BOOL); st.push_back(a); break;            // NEWFALSE
            case 'N': st.push_back(mk(Val::NONE)); break;
            case 'c': {  // GLOBAL: recorded as a name, never resolved
                std::string m, nm;
                if (!line(&m) || !line(&nm)) return bad("GLOBAL");
                a = mk(Val::GLOBAL);
                a->s = m + " " + nm;
                st.push_back(a);
                break;
            }
            case 'q': if (!need(1) || st.empty()) return bad("BINPUT"); memo[p[i]] = st.back(); i += 1; break;
            case 'r': if (!need(4) || st.empty()) return bad("LONG_BINPUT"); memo[rd32(p + i)] = st.back(); i += 4; break;
            case 0x94: if (st.empty()) return bad("MEMOIZE"); memo[memo.size()] = st.back(); break;
            case 'h':
                if (!need(1) || !memo.count(p[i])) return bad("BINGET");
                st.push_back(memo[p[i]]);
                i += 1;
                break;
            case 'j':
                if (!need(4) || !memo.count(rd32(p + i))) return bad("LONG_BINGET");
                st.push_back(memo[rd32(p + i)]);
                i += 4;
                break;
            case '(': marks.push_back(st.size()); break;
            case 't':
                if (!since_mark(&xs)) return bad("TUPLE");
                a = mk(Val::TUPLE);
                a->items = xs;
                st.push_back(a);
                break;
            case ')': st.push_back(mk(Val::TUPLE)); break;
            case 0x85: case 0x86: case 0x87: {  // TUPLE1..3
                const size_t k = op - 0x84u;
                if (st.size() < k) return bad("TUPLEn");
                a = mk(Val::TUPLE);
                a->items.assign(st.end() - (long)k, st.end());
                st.resize(st.size() - k);
                st.push_back(a);
                break;
            }
            case '}': st.push_back(mk(Val::DICT)); break;
            case ']': st.push_back(mk(Val::LIST)); break;
            case 'u':  // SETITEMS
                if (!since_mark(&xs) || st.empty() || (xs.size() & 1)) return bad("SETITEMS");
                if (st.back()->k == Val::DICT) st.back()->items.insert(st.back()->items.end(), xs.begin(), xs.end());
                break;
            case 's':  // SETITEM
                if (!pop(&b) || !pop(&a) || st.empty()) return bad("SETITEM");
                if (st.back()->k == Val::DICT) st.back()->items.push_back(a), st.back()->items.push_back(b);
                break;
            case 'e':  // APPENDS
                if (!since_mark(&xs) || st.empty()) return bad("APPENDS");
                if (st.back()->k == Val::LIST) st.back()->items.insert(st.back()->items.end(), xs.begin(), xs.end());
                break;
            case 'a':  // APPEND
                if (!pop(&a) || st.empty()) return bad("APPEND");
                if (st.back()->k == Val::LIST) st.back()->items.push_back(a);
                break;
            case 'Q':  // BINPERSID
                if (!pop(&a)) return bad("BINPERSID");
                b = mk(Val::PERSID);
                b->args = a;
                st.push_back(b);
                break;
            case 'R': case 0x81:  // REDUCE / NEWOBJ: recorded as a call, never made
                if (!pop(&b) || !pop(&a)) return bad("REDUCE");
                c = mk(Val::CALL);
                c->callee = a;
                c->args = b;
                st.push_back(c);
                break;
            case 'b':  // BUILD
                if (!pop(&a) || st.empty()) return bad("BUILD");
                if (st.back()->k == Val::CALL) st.back()->state = a;
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

bool is_global(const V& v, const char* name) { return v && v->k == Val::GLOBAL && v->s == name; }

// name -> _rebuild_tensor_v2 record, from every dict reachable from the root (the module's state)
int find_tensors(const V& v, std::map<std::string, TensorRec>& out, int depth = 0) {
    if (!v || depth > 64) return 0;
    if (v->k == Val::DICT) {
        for (size_t j = 0; j + 1 < v->items.size(); j += 2) {
            const V& key = v->items[j];
            const V& val = v->items[j + 1];
            if (key->k == Val::STR && val->k == Val::CALL && is_global(val->callee, "torch._utils _rebuild_tensor_v2")) {
                const V& a = val->args;  // (persid, offset, shape, stride, requires_grad, hooks)
                if (!a || a->k != Val::TUPLE || a->items.size() < 4 || a->items[0]->k != Val::PERSID)
                    return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: tensor '%s': unexpected record", key->s.c_str());
                const V& pers = a->items[0]->args;  // ('storage', <dtype storage>, key, location, numel)
                if (!pers || pers->k != Val::TUPLE || pers->items.size() < 3 || pers->items[2]->k != Val::STR)
                    return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: tensor '%s': unexpected storage record", key->s.c_str());
                if (!is_global(pers->items[1], "torch FloatStorage"))
                    return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: tensor '%s': storage %s (fp32 only)", key->s.c_str(),
                                       pers->items[1]->s.c_str());
                TensorRec r;
                r.key = pers->items[2]->s;
                if (a->items[1]->k != Val::INT) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: '%s': bad offset", key->s.c_str());
                r.offset = a->items[1]->i;
                for (int w = 2; w <= 3; ++w) {
                    if (a->items[w]->k != Val::TUPLE) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: '%s': bad shape", key->s.c_str());
                    for (const V& d : a->items[w]->items) {
                        if (d->k != Val::INT) return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: '%s': bad shape", key->s.c_str());
                        (w == 2 ? r.shape : r.stride).push_back(d->i);
                    }
                }
                if (r.shape.size() != r.stride.size() || r.shape.size() > 6)
                    return oaz_set_err(OAZ_ERR_WEIGHTS, "ot: '%s': bad shape/stride", key->s.c_str());
                out[key->s] = r;
            } else if (int rc = find_tensors(val, out, depth + 1)) {
                return rc;
            }
        }
    } else if (v->k == Val::TUPLE || v->k == Val::LIST) {
        for (const V& x : v->items)
            if (int rc = find_tensors(x, out, depth + 1)) return rc;
    } else if (v->k == Val::CALL) {
        if (int rc = find_tensors(v->args, out, depth + 1)) return rc;
        if (int rc = find_tensors(v->state, out, depth + 1)) return rc;
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
    V top;
    if (int rc = unpickle(&f[pkl->data_off], (size_t)pkl->size, &top)) return rc;
    std::map<std::string, TensorRec> recs;
    if (int rc = find_tensors(top, recs)) return rc;
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
