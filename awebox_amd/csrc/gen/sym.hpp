// Tracing scalar and sparse symbolic forward differentiation for generating straight-line
// node-Jacobian code (host only; build-time tool).
//
// The reference obtains J_g by CasADi's symbolic AD on the expanded SX graph of the collocation
// NLP and evaluates the result in CasADi's SX virtual machine (awebox/opti/preparation.py:366-400,
// ocp/nlp.py:77-161).  The same idea, specialised to one collocation node: the templated node
// model (ap2_model.hpp) is run once on `Sym`, which records every operation in a hash-consed tape
// (common subexpressions merge, constants fold, x*1 / x+0 / x*0 simplify).  `forward_grads`
// then propagates *sparse* symbolic tangents through the tape -- one tangent per (node,
// direction) that is structurally non-zero -- and `emit` writes the value and tangent nodes the
// outputs need as straight-line C++ (one statement per operation), ordered so that each tangent
// is computed right after the value it belongs to.  The result runs one thread per collocation
// node on the GPU and issues only the algorithmic flops, instead of one dual number per
// colour lane.
#pragma once

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <climits>
#include <cstring>
#include <functional>
#include <map>
#include <cstdlib>
#include <set>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace awe {

enum class Op : uint8_t { Const, Input, Th, Cs, Extra, Add, Sub, Mul, Neg, Rcp, Sqrt, Exp, Log, Sin, Cos };

struct SNode {
    Op op;
    int a, b;       // operands (-1: none)
    double c;       // constant value (Const)
    int idx;        // input / parameter index
    double val;     // value recorded at trace time (parameters: for structural reads only)
};

class Tape {
  public:
    std::vector<SNode> n;
    std::vector<int> owner;        // emission group: the value node whose tangents created it

    int cnst(double v) { return make(Op::Const, -1, -1, v, 0, v); }
    int leaf(Op op, int idx, double val = 0.0) { return make(op, -1, -1, 0.0, idx, val); }
    bool is_const(int id, double* v = nullptr) const {
        if (n[id].op != Op::Const) return false;
        if (v) *v = n[id].c;
        return true;
    }
    bool is_c(int id, double x) const { double v; return is_const(id, &v) && v == x && !std::signbit(v - x); }

    // Negations are pushed outward (all rewrites are exact in IEEE arithmetic): a + (-b) = a - b,
    // a - (-b) = a + b, (-a) b = -(a b), 1 / (-a) = -(1 / a).  They end up absorbed by additions or at
    // the stores, so that the emitted code has (almost) no separate negation for the compiler to
    // fold back into a multiply at the consumer's position, which would stretch the multiply's
    // operands' live ranges.
    bool is_neg(int id) const { return n[id].op == Op::Neg; }
    int add(int a, int b) {
        double va, vb;
        const bool ca = is_const(a, &va), cb = is_const(b, &vb);
        if (ca && cb) return cnst(va + vb);
        if (ca && va == 0.0) return b;
        if (cb && vb == 0.0) return a;
        if (is_neg(a) && is_neg(b)) return neg(add(n[a].a, n[b].a));
        if (is_neg(b)) return sub(a, n[b].a);
        if (is_neg(a)) return sub(b, n[a].a);
        if (a > b) std::swap(a, b);
        return make(Op::Add, a, b);
    }
    int sub(int a, int b) {
        double va, vb;
        const bool ca = is_const(a, &va), cb = is_const(b, &vb);
        if (ca && cb) return cnst(va - vb);
        if (cb && vb == 0.0) return a;
        if (ca && va == 0.0) return neg(b);
        if (is_neg(b)) return add(a, n[b].a);
        if (is_neg(a)) return neg(add(n[a].a, b));
        return make(Op::Sub, a, b);
    }
    int mul(int a, int b) {
        double va, vb;
        const bool ca = is_const(a, &va), cb = is_const(b, &vb);
        if (ca && cb) return cnst(va * vb);
        if (is_neg(a) && is_neg(b)) return mul(n[a].a, n[b].a);
        if (is_neg(a)) return neg(mul(n[a].a, b));
        if (is_neg(b)) return neg(mul(a, n[b].a));
        if (ca && va < 0.0 && va != -1.0) return neg(mul(cnst(-va), b));
        if (cb && vb < 0.0 && vb != -1.0) return neg(mul(a, cnst(-vb)));
        if (ca) {
            if (va == 0.0) return cnst(0.0);
            if (va == 1.0) return b;
            if (va == -1.0) return neg(b);
        }
        if (cb) {
            if (vb == 0.0) return cnst(0.0);
            if (vb == 1.0) return a;
            if (vb == -1.0) return neg(a);
        }
        if (a > b) std::swap(a, b);
        return make(Op::Mul, a, b);
    }
    int neg(int a) {
        double va;
        if (is_const(a, &va)) return cnst(-va);
        if (n[a].op == Op::Neg) return n[a].a;
        return make(Op::Neg, a, -1);
    }
    int rcp(int a) {
        double va;
        if (is_const(a, &va)) return cnst(1.0 / va);
        if (is_neg(a)) return neg(rcp(n[a].a));
        return make(Op::Rcp, a, -1);
    }
    int div(int a, int b) {
        double vb;
        if (is_const(b, &vb)) return mul(a, cnst(1.0 / vb));
        return mul(a, rcp(b));
    }
    int un(Op op, int a) {
        double va;
        if (is_const(a, &va)) {
            switch (op) {
                case Op::Sqrt: return cnst(std::sqrt(va));
                case Op::Exp: return cnst(std::exp(va));
                case Op::Log: return cnst(std::log(va));
                case Op::Sin: return cnst(std::sin(va));
                case Op::Cos: return cnst(std::cos(va));
                default: break;
            }
        }
        return make(op, a, -1);
    }

    int group = -1;   // current emission group (set by forward_grads)
    bool extra_call = false;   // emit extra leaves as ex(i) (an accessor) instead of variables ex<i>

  private:
    struct Key {
        uint8_t op; int a, b, idx; uint64_t c;
        bool operator==(const Key& o) const { return op == o.op && a == o.a && b == o.b && idx == o.idx && c == o.c; }
    };
    struct KeyHash {
        size_t operator()(const Key& k) const {
            uint64_t h = k.op;
            h = h * 0x9E3779B97F4A7C15ull ^ (uint64_t)(uint32_t)k.a;
            h = h * 0x9E3779B97F4A7C15ull ^ (uint64_t)(uint32_t)k.b;
            h = h * 0x9E3779B97F4A7C15ull ^ (uint64_t)(uint32_t)k.idx;
            h = h * 0x9E3779B97F4A7C15ull ^ k.c;
            return (size_t)(h ^ (h >> 29));
        }
    };
    std::unordered_map<Key, int, KeyHash> hc_;

    int make(Op op, int a, int b, double c = 0.0, int idx = 0, double val = 0.0) {
        uint64_t cb = 0;
        std::memcpy(&cb, &c, sizeof(cb));
        Key k{(uint8_t)op, a, b, idx, cb};
        auto it = hc_.find(k);
        if (it != hc_.end()) return it->second;
        const int id = (int)n.size();
        n.push_back(SNode{op, a, b, c, idx, val});
        // emitted with the latest of: its creator's group and its operands' groups
        int own = group < 0 ? id : group;
        if (a >= 0) own = std::max(own, owner[a]);
        if (b >= 0) own = std::max(own, owner[b]);
        owner.push_back(own);
        hc_.emplace(k, id);
        return id;
    }
};

inline Tape*& active_tape() {
    static Tape* t = nullptr;
    return t;
}

struct Sym {
    int id;
    Sym() : id(active_tape()->cnst(0.0)) {}
    Sym(double v) : id(active_tape()->cnst(v)) {}
    static Sym of(int i) { Sym s(0.0); s.id = i; return s; }
};

inline Tape& T_() { return *active_tape(); }
inline Sym operator+(Sym a, Sym b) { return Sym::of(T_().add(a.id, b.id)); }
inline Sym operator-(Sym a, Sym b) { return Sym::of(T_().sub(a.id, b.id)); }
inline Sym operator*(Sym a, Sym b) { return Sym::of(T_().mul(a.id, b.id)); }
inline Sym operator/(Sym a, Sym b) { return Sym::of(T_().div(a.id, b.id)); }
inline Sym operator-(Sym a) { return Sym::of(T_().neg(a.id)); }
inline Sym operator+(Sym a, double b) { return a + Sym(b); }
inline Sym operator+(double a, Sym b) { return Sym(a) + b; }
inline Sym operator-(Sym a, double b) { return a - Sym(b); }
inline Sym operator-(double a, Sym b) { return Sym(a) - b; }
inline Sym operator*(Sym a, double b) { return a * Sym(b); }
inline Sym operator*(double a, Sym b) { return Sym(a) * b; }
inline Sym operator/(Sym a, double b) { return a / Sym(b); }
inline Sym operator/(double a, Sym b) { return Sym(a) / b; }
inline Sym& operator+=(Sym& a, Sym b) { a = a + b; return a; }
inline Sym& operator-=(Sym& a, Sym b) { a = a - b; return a; }
inline Sym& operator*=(Sym& a, Sym b) { a = a * b; return a; }
inline Sym sqrt(Sym a) { return Sym::of(T_().un(Op::Sqrt, a.id)); }
inline Sym exp(Sym a) { return Sym::of(T_().un(Op::Exp, a.id)); }
inline Sym log(Sym a) { return Sym::of(T_().un(Op::Log, a.id)); }
inline Sym sin(Sym a) { return Sym::of(T_().un(Op::Sin, a.id)); }
inline Sym cos(Sym a) { return Sym::of(T_().un(Op::Cos, a.id)); }
// structural integer read from a model constant: the value recorded at trace time
inline int structural(Sym a) {
    const SNode& s = T_().n[a.id];
    return (int)(s.op == Op::Const ? s.c : s.val);
}

// ---- sparse forward tangents ---------------------------------------------------------------
using SparseGrad = std::vector<std::pair<int, int>>;   // (direction, tape node), by direction

// Propagates the tangents of the first n0 tape nodes; `seed(input index)` gives an input's
// tangent.  Nodes created while differentiating value node i join emission group i.
inline std::vector<SparseGrad> forward_grads(Tape& t, int n0, const std::function<SparseGrad(int)>& seed) {
    std::vector<SparseGrad> G(n0);
    auto merge = [&t](const SparseGrad& x, const SparseGrad& y, const std::function<int(int, int)>& both,
                    const std::function<int(int)>& only_x, const std::function<int(int)>& only_y) {
        SparseGrad r;
        size_t i = 0, j = 0;
        while (i < x.size() || j < y.size()) {
            if (j == y.size() || (i < x.size() && x[i].first < y[j].first)) {
                r.emplace_back(x[i].first, only_x(x[i].second)); ++i;
            } else if (i == x.size() || y[j].first < x[i].first) {
                r.emplace_back(y[j].first, only_y(y[j].second)); ++j;
            } else {
                r.emplace_back(x[i].first, both(x[i].second, y[j].second)); ++i; ++j;
            }
        }
        r.erase(std::remove_if(r.begin(), r.end(), [&](const std::pair<int, int>& p) { return t.is_c(p.second, 0.0); }),
                r.end());
        return r;
    };
    auto scale = [&](const SparseGrad& x, const std::function<int(int)>& f) {
        SparseGrad r;
        for (auto& p : x) {
            const int v = f(p.second);
            if (!t.is_c(v, 0.0)) r.emplace_back(p.first, v);
        }
        return r;
    };
    auto id = [](int x) { return x; };
    for (int i = 0; i < n0; ++i) {
        t.group = i;
        const SNode s = t.n[i];
        switch (s.op) {
            case Op::Const: case Op::Th: case Op::Cs: case Op::Extra: break;
            case Op::Input: G[i] = seed(s.idx); break;
            case Op::Add:
                G[i] = merge(G[s.a], G[s.b], [&](int x, int y) { return t.add(x, y); }, id, id);
                break;
            case Op::Sub:
                G[i] = merge(G[s.a], G[s.b], [&](int x, int y) { return t.sub(x, y); }, id,
                             [&](int y) { return t.neg(y); });
                break;
            case Op::Mul:
                // (a b)' = a' b + a b'  (the order of the dual-number product, scalar.hpp)
                G[i] = merge(G[s.a], G[s.b], [&](int x, int y) { return t.add(t.mul(x, s.b), t.mul(s.a, y)); },
                             [&](int x) { return t.mul(x, s.b); }, [&](int y) { return t.mul(s.a, y); });
                break;
            case Op::Neg: G[i] = scale(G[s.a], [&](int x) { return t.neg(x); }); break;
            case Op::Rcp: {
                if (G[s.a].empty()) break;
                const int f = t.neg(t.mul(i, i));
                G[i] = scale(G[s.a], [&](int x) { return t.mul(x, f); });
                break;
            }
            case Op::Sqrt: {
                if (G[s.a].empty()) break;
                const int f = t.mul(t.cnst(0.5), t.rcp(i));
                G[i] = scale(G[s.a], [&](int x) { return t.mul(x, f); });
                break;
            }
            case Op::Exp:
                G[i] = scale(G[s.a], [&](int x) { return t.mul(i, x); });
                break;
            case Op::Log: {
                if (G[s.a].empty()) break;
                const int f = t.rcp(s.a);
                G[i] = scale(G[s.a], [&](int x) { return t.mul(x, f); });
                break;
            }
            case Op::Sin: {
                if (G[s.a].empty()) break;
                const int f = t.un(Op::Cos, s.a);
                G[i] = scale(G[s.a], [&](int x) { return t.mul(f, x); });
                break;
            }
            case Op::Cos: {
                if (G[s.a].empty()) break;
                const int f = t.neg(t.un(Op::Sin, s.a));
                G[i] = scale(G[s.a], [&](int x) { return t.mul(f, x); });
                break;
            }
        }
    }
    t.group = -1;
    return G;
}

// ---- emission --------------------------------------------------------------------------------
struct Store {
    int node;        // tape node stored
    int kind;        // 0 value row val[row], 1 tangent tan[slot], 2 dbp[dir], 3 obv[row]
    int row, dir;
    int slot = -1;   // tangent-buffer index (kind 1), assigned by emit
};

struct EmitStats {
    int ops = 0, flops = 0, transcendental = 0, loads = 0, n_tan = 0, n_zero_tan = 0, max_live = 0;
};

inline std::string hexlit(double v) {
    char buf[64];
    if (v == 0.0) return std::signbit(v) ? "-0.0" : "0.0";
    std::snprintf(buf, sizeof(buf), "%a", v);
    return buf;
}


// Negations are not emitted as statements: a consumer reads (-x) (a free source modifier of the
// FP64 ALU), so for scheduling and liveness an operand that is a negation stands for its operand.
inline int res(const Tape& t, int v) { return (v >= 0 && t.n[v].op == Op::Neg) ? t.n[v].a : v; }

// List scheduling for register pressure.  `order` is a valid topological order (the baseline);
// nodes are re-emitted greedily: among the ready nodes, the one that frees the most live values
// (operands whose last consumer it is, net of the value it defines, which counts as free when
// only stores use it) goes first, ties broken by the baseline position.  Loads therefore wait
// until their consumer can run, and a chain is finished before the next one is opened.
using Operands = std::array<int, 3>;   // resolved operands of an emitted node (-1: none)

inline std::vector<int> pressure_schedule(const Tape& t, const std::vector<int>& order,
                                          const std::vector<Operands>& ops) {
    const int N = (int)t.n.size();
    std::vector<int> base(N, -1);
    for (size_t i = 0; i < order.size(); ++i) base[order[i]] = (int)i;
    auto in_sched = [&](int v) { return v >= 0 && base[v] >= 0; };
    // distinct scheduled operands of v (a node may use one operand twice: x * x)
    auto dops = [&](int v) {
        std::vector<int> r;
        for (int o : ops[v])
            if (in_sched(o) && std::find(r.begin(), r.end(), o) == r.end()) r.push_back(o);
        return r;
    };
    std::vector<std::vector<int>> users(N);
    std::vector<int> remaining(N, 0), pending(N, 0);
    for (int v : order)
        for (int o : dops(v)) users[o].push_back(v);
    for (int v : order) {
        remaining[v] = (int)users[v].size();
        pending[v] = (int)dops(v).size();
    }
    auto score = [&](int v) {
        int freed = 0;
        for (int o : dops(v)) if (remaining[o] == 1) ++freed;
        const int def = users[v].empty() ? 0 : 1;    // stored-only values die at once
        return freed - def;
    };
    // ready set ordered by (score desc, baseline asc); scores change only for the ready users of
    // operands whose remaining count drops to 1, which are re-inserted
    std::vector<int> out;
    out.reserve(order.size());
    std::vector<char> done(N, 0), ready(N, 0);
    std::vector<int> cur_score(N, 0);
    struct Cmp {
        bool operator()(const std::pair<int, int>& x, const std::pair<int, int>& y) const {
            return x.first != y.first ? x.first > y.first : x.second < y.second;
        }
    };
    std::set<std::pair<int, int>, Cmp> rs;   // (score, baseline position)
    auto push = [&](int v) {
        ready[v] = 1;
        cur_score[v] = score(v);
        rs.insert({cur_score[v], base[v]});
    };
    for (int v : order)
        if (pending[v] == 0) push(v);
    while (!rs.empty()) {
        const int v = order[rs.begin()->second];
        rs.erase(rs.begin());
        done[v] = 1;
        out.push_back(v);
        auto consume = [&](int o) {
            if (!in_sched(o)) return;
            remaining[o]--;
            if (remaining[o] == 1) {
                for (int u : users[o])
                    if (ready[u] && !done[u]) {
                        rs.erase({cur_score[u], base[u]});
                        cur_score[u] = score(u);
                        rs.insert({cur_score[u], base[u]});
                    }
            }
        };
        for (int o : dops(v)) consume(o);
        for (int u : users[v])
            if (--pending[u] == 0) push(u);
    }
    return out;
}

// Writes the body of a straight-line function: every tape node the stores need, in emission-group
// order (a value, then the tangents it created), each store right after its node.  Tangent
// stores take consecutive slots in the order they are executed, so one thread's stores run
// through memory sequentially.  Names: in(i) inputs, th[i] / cst[i] parameters, ex<i> extras,
// val[r] / tan[s] outputs.
inline std::string emit(Tape& t, std::vector<Store>& stores, EmitStats& st, bool schedule = true,
                        int barrier_every = 0, bool opaque = false, int slot_base_in = 0, bool fuse = true) {
    int slot_base = slot_base_in;
    const bool keep_all = std::getenv("AWE_GEN_KEEP_ALL") != nullptr;
    const int N = (int)t.n.size();
    std::vector<char> live(N, 0);
    std::vector<int> stack;
    for (auto& s : stores) stack.push_back(s.node);
    while (!stack.empty()) {
        const int v = stack.back();
        stack.pop_back();
        if (live[v]) continue;
        live[v] = 1;
        if (t.n[v].a >= 0) stack.push_back(t.n[v].a);
        if (t.n[v].b >= 0) stack.push_back(t.n[v].b);
    }
    // emission key: (group, index); a leaf (input, parameter) takes the key of its first consumer,
    // so that loads are issued where they are needed instead of all at the top
    std::vector<std::pair<int, int>> key(N);
    for (int v = 0; v < N; ++v) key[v] = {t.owner[v], v};
    auto is_leaf = [&](int v) {
        const Op op = t.n[v].op;
        return op == Op::Input || op == Op::Th || op == Op::Cs || op == Op::Extra;
    };
    std::vector<std::pair<int, int>> first_use(N, {INT32_MAX, INT32_MAX});
    for (int v = 0; v < N; ++v) {
        if (!live[v] || t.n[v].op == Op::Neg) continue;
        for (int o : {res(t, t.n[v].a), res(t, t.n[v].b)})
            if (o >= 0 && is_leaf(o)) first_use[o] = std::min(first_use[o], key[v]);
    }
    for (int v = 0; v < N; ++v)
        if (live[v] && is_leaf(v) && first_use[v].first != INT32_MAX) key[v] = {first_use[v].first, first_use[v].second - 1};
    std::vector<int> order;
    for (int v = 0; v < N; ++v)
        if (live[v] && t.n[v].op != Op::Const && t.n[v].op != Op::Neg) order.push_back(v);
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return key[x] < key[y]; });
    // operands as emitted: negations resolved; a multiply used only by one addition or
    // subtraction is fused into it (an explicit fma: one rounding, and the multiply's operands are
    // consumed where the sum is formed, which the schedule then accounts for)
    std::vector<Operands> ops(N, Operands{-1, -1, -1});
    struct Fused { int m = -1, other = -1; bool neg_prod = false, neg_other = false; };
    std::vector<Fused> fz(N);
    {
        std::vector<int> uses(N, 0);
        for (int v : order) {
            std::vector<int> seen;
            for (int o : {res(t, t.n[v].a), res(t, t.n[v].b)})
                if (o >= 0 && std::find(seen.begin(), seen.end(), o) == seen.end()) { seen.push_back(o); uses[o]++; }
        }
        for (auto& x : stores) uses[res(t, x.node)]++;
        std::vector<char> absorbed(N, 0);
        for (int v : order) {
            const SNode& s = t.n[v];
            ops[v] = Operands{res(t, s.a), res(t, s.b), -1};
            if (!fuse || (s.op != Op::Add && s.op != Op::Sub)) continue;
            // v = a + b or a - b; try the operand slots in turn
            for (int slot = 0; slot < 2; ++slot) {
                const int raw = slot == 0 ? s.a : s.b, oraw = slot == 0 ? s.b : s.a;
                const int m = res(t, raw);
                if (t.n[m].op != Op::Mul || uses[m] != 1 || absorbed[m] || m == res(t, oraw)) continue;
                Fused f;
                f.m = m;
                f.other = oraw;
                f.neg_prod = (raw != m) != (s.op == Op::Sub && slot == 1);
                f.neg_other = s.op == Op::Sub && slot == 0;
                fz[v] = f;
                absorbed[m] = 1;
                ops[v] = Operands{res(t, t.n[m].a), res(t, t.n[m].b), res(t, oraw)};
                break;
            }
        }
        std::vector<int> kept;
        for (int v : order) if (!absorbed[v]) kept.push_back(v);
        order.swap(kept);
    }
    if (schedule) order = pressure_schedule(t, order, ops);
    std::vector<int> pos(N, -1);
    for (size_t i = 0; i < order.size(); ++i) pos[order[i]] = (int)i;
    // stores of constant nodes (zero tangents) go first, the others after their node
    std::vector<std::vector<int>> after(order.size());
    std::vector<int> early;
    for (size_t s = 0; s < stores.size(); ++s) {
        const int v = res(t, stores[s].node);
        if (t.n[v].op == Op::Const) early.push_back((int)s);
        else after[pos[v]].push_back((int)s);
    }
    {   // register pressure of this order: values live from definition to last use
        std::vector<int> last(N, -1);
        for (size_t i = 0; i < order.size(); ++i)
            for (int o : ops[order[i]])
                if (o >= 0 && pos[o] >= 0) last[o] = std::max(last[o], (int)i);
        for (size_t i = 0; i < order.size(); ++i)
            for (int sidx : after[i]) {
                const int v = res(t, stores[sidx].node);
                last[v] = std::max(last[v], (int)i);
            }
        std::vector<int> delta(order.size() + 1, 0);
        for (size_t i = 0; i < order.size(); ++i) {
            const int v = order[i];
            if (last[v] < 0) continue;
            delta[i] += 1;
            delta[last[v] + 1] -= 1;
        }
        int cur = 0, at = 0;
        for (size_t i = 0; i < order.size(); ++i) {
            cur += delta[i];
            if (cur > st.max_live) { st.max_live = cur; at = (int)i; }
        }
        if (std::getenv("AWE_GEN_DEBUG")) {   // what is live at the high-water mark
            std::map<int, int> by_owner;
            int nval = 0;
            for (int j = 0; j <= at; ++j) {
                const int v = order[j];
                if (last[v] >= at) {
                    by_owner[t.owner[v]]++;
                    if (t.owner[v] == v) ++nval;
                }
            }
            std::fprintf(stderr, "peak %d at %d/%zu: %d values, %zu groups:", st.max_live, at, order.size(), nval,
                         by_owner.size());
            for (auto& kv : by_owner) std::fprintf(stderr, " %d:%d", kv.first, kv.second);
            std::fprintf(stderr, "\n");
        }
    }
    std::string out;
    char buf[256];
    auto ref = [&](int v) -> std::string {
        if (t.n[v].op == Op::Const) return "(" + hexlit(t.n[v].c) + ")";
        if (t.n[v].op == Op::Neg) return "(-v" + std::to_string(t.n[v].a) + ")";
        return "v" + std::to_string(v);
    };
    int& next_slot = slot_base;
    // a strip after the first re-reads its leaves through an opaque copy, so that the compiler
    // recomputes the strip's values instead of keeping the first strip's alive
    auto opq = [&](const std::string& x) { return opaque ? "AWE_GEN_OPAQUE(" + x + ")" : x; };
    auto put_store = [&](int s) {
        Store& x = stores[s];
        if (x.kind == 0) {
            std::snprintf(buf, sizeof(buf), "    val[%d] = %s;\n", x.row, ref(x.node).c_str());
        } else if (x.kind == 2) {
            std::snprintf(buf, sizeof(buf), "    dbp[%d] = %s;\n", x.dir, ref(x.node).c_str());
        } else if (x.kind == 3) {
            std::snprintf(buf, sizeof(buf), "    obv[%d] = %s;\n", x.row, ref(x.node).c_str());
        } else {
            x.slot = next_slot++;
            std::snprintf(buf, sizeof(buf), "    tan[%d * TS] = %s;\n", x.slot, ref(x.node).c_str());
            st.n_tan++;
            if (t.n[x.node].op == Op::Const) st.n_zero_tan++;
        }
        out += buf;
    };
    for (int s : early) put_store(s);
    for (size_t i = 0; i < order.size(); ++i) {
        const int v = order[i];
        const SNode& s = t.n[v];
        std::string e;
        switch (s.op) {
            case Op::Input: e = opq("in(" + std::to_string(s.idx) + ")"); st.loads++; break;
            case Op::Th: e = opq("th[" + std::to_string(s.idx) + "]"); st.loads++; break;
            case Op::Cs: e = opq("cst[" + std::to_string(s.idx) + "]"); st.loads++; break;
            case Op::Extra:
                e = opq(t.extra_call ? "ex(" + std::to_string(s.idx) + ")" : "ex" + std::to_string(s.idx));
                break;
            case Op::Add:
            case Op::Sub:
                if (fz[v].m >= 0) {
                    const SNode& m = t.n[fz[v].m];
                    auto sg = [](bool neg, const std::string& x) { return neg ? "(-" + x + ")" : x; };
                    e = "__builtin_fma(" + sg(fz[v].neg_prod, ref(m.a)) + ", " + ref(m.b) + ", " +
                        sg(fz[v].neg_other, ref(fz[v].other)) + ")";
                    st.flops += 2;
                    break;
                }
                e = ref(s.a) + (s.op == Op::Add ? " + " : " - ") + ref(s.b);
                st.flops++;
                break;
            case Op::Mul: e = ref(s.a) + " * " + ref(s.b); if (std::getenv("AWE_GEN_KEEP_MUL")) e = "AWE_GEN_KEEP(" + e + ")"; st.flops++; break;
            case Op::Neg: break;   // folded into its consumers (ref)
            case Op::Rcp: e = "awe::rcp(" + ref(s.a) + ")"; st.flops++; break;
            case Op::Sqrt: e = "::sqrt(" + ref(s.a) + ")"; st.transcendental++; break;
            case Op::Exp: e = "::exp(" + ref(s.a) + ")"; st.transcendental++; break;
            case Op::Log: e = "::log(" + ref(s.a) + ")"; st.transcendental++; break;
            case Op::Sin: e = "::sin(" + ref(s.a) + ")"; st.transcendental++; break;
            case Op::Cos: e = "::cos(" + ref(s.a) + ")"; st.transcendental++; break;
            case Op::Const: break;
        }
        st.ops++;
        if (keep_all && (s.op == Op::Add || s.op == Op::Sub || s.op == Op::Rcp)) e = "AWE_GEN_KEEP(" + e + ")";
        out += "    const double v" + std::to_string(v) + " = " + e + ";\n";
        if (barrier_every > 0 && st.ops % barrier_every == 0) out += "    AWE_GEN_FENCE();\n";
        for (int sidx : after[i]) put_store(sidx);
    }
    return out;
}

}  // namespace awe
