// Native host-side prioritized-replay core (C++17, pybind11).
//
// Behavioural model: reference memory.py:10-143 (SegmentTree / SumSegmentTree /
// MinSegmentTree) and memory.py:208-320 (PrioritizedReplayBuffer priority logic).
// The reference walks Python lists under one asyncio lock (origin_repo/replay.py:92-143);
// here the trees are flat double arrays and every batch operation (add, update,
// stratified sample, IS weights) is a single native call, so the Python layer never
// loops per transition.
//
// Numerics: all tree nodes are IEEE double and every ancestor is recomputed as
// op(left, right) exactly like the reference, so sums / prefix descents are bitwise
// identical to the reference for the same inputs (build with -ffp-contract=off).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

enum class TreeOp { Sum, Min };

class Tree {
 public:
  Tree(int64_t capacity, TreeOp op) : cap_(capacity), op_(op) {
    if (capacity <= 0 || (capacity & (capacity - 1)) != 0)
      throw std::invalid_argument("capacity must be positive and a power of 2.");
    neutral_ = op == TreeOp::Sum ? 0.0 : std::numeric_limits<double>::infinity();
    v_.assign(static_cast<size_t>(2 * capacity), neutral_);
  }

  inline double combine(double a, double b) const {
    // reference: operator.add / builtin min (min returns the first arg on ties)
    if (op_ == TreeOp::Sum) return a + b;
    return (b < a) ? b : a;
  }

  void set(int64_t idx, double val) {
    if (idx < 0 || idx >= cap_) throw std::out_of_range("tree index out of range");
    int64_t i = idx + cap_;
    v_[i] = val;
    i >>= 1;
    while (i >= 1) {
      v_[i] = combine(v_[2 * i], v_[2 * i + 1]);
      i >>= 1;
    }
  }

  double get(int64_t idx) const {
    if (idx < 0 || idx >= cap_) throw std::out_of_range("tree index out of range");
    return v_[cap_ + idx];
  }

  // Inclusive range reduction with the reference's recursion order (memory.py:39-52).
  double reduce_helper(int64_t start, int64_t end, int64_t node, int64_t ns, int64_t ne) const {
    if (start == ns && end == ne) return v_[node];
    int64_t mid = (ns + ne) / 2;
    if (end <= mid) return reduce_helper(start, end, 2 * node, ns, mid);
    if (mid + 1 <= start) return reduce_helper(start, end, 2 * node + 1, mid + 1, ne);
    return combine(reduce_helper(start, mid, 2 * node, ns, mid),
                   reduce_helper(mid + 1, end, 2 * node + 1, mid + 1, ne));
  }

  // Python-facing reduce(start, end): `end` exclusive, None -> capacity, negative wraps
  // (memory.py:54-74).
  double reduce(int64_t start, py::object end_obj) const {
    int64_t end = end_obj.is_none() ? cap_ : end_obj.cast<int64_t>();
    if (end < 0) end += cap_;
    end -= 1;
    if (end < start) return neutral_;  // the reference recurses forever here; we return the identity
    return reduce_helper(start, end, 1, 0, cap_ - 1);
  }

  int64_t find_prefixsum_idx(double prefixsum) const {
    int64_t idx = 1;
    while (idx < cap_) {
      if (v_[2 * idx] > prefixsum) {
        idx = 2 * idx;
      } else {
        prefixsum -= v_[2 * idx];
        idx = 2 * idx + 1;
      }
    }
    return idx - cap_;
  }

  int64_t capacity() const { return cap_; }
  double root() const { return v_[1]; }
  const std::vector<double>& values() const { return v_; }

 private:
  int64_t cap_;
  TreeOp op_;
  double neutral_;
  std::vector<double> v_;
};

template <typename T>
const T* data1d(const py::array_t<T, py::array::c_style | py::array::forcecast>& a) {
  if (a.ndim() != 1) throw std::invalid_argument("expected a 1-D array");
  return a.data();
}

// PER core = sum tree + min tree + alpha + running max priority (memory.py:208-320).
class PERCore {
 public:
  PERCore(int64_t size, double alpha) : alpha_(alpha), max_priority_(1.0) {
    if (alpha < 0) throw std::invalid_argument("alpha must be >= 0");
    int64_t cap = 1;
    while (cap < size) cap *= 2;
    sum_ = std::make_unique<Tree>(cap, TreeOp::Sum);
    min_ = std::make_unique<Tree>(cap, TreeOp::Min);
  }

  // Insert with max-priority (PrioritizedReplayBuffer.add, memory.py:235-240).
  void add_max(py::array_t<int64_t, py::array::c_style | py::array::forcecast> idx) {
    const int64_t* p = data1d(idx);
    double v = std::pow(max_priority_, alpha_);
    for (py::ssize_t i = 0; i < idx.shape(0); ++i) {
      sum_->set(p[i], v);
      min_->set(p[i], v);
    }
  }

  // Insert with actor-computed priorities (CustomPrioritizedReplayBuffer.add, memory.py:334-346).
  void add_with_priority(py::array_t<int64_t, py::array::c_style | py::array::forcecast> idx,
                         py::array_t<double, py::array::c_style | py::array::forcecast> prio) {
    const int64_t* pi = data1d(idx);
    const double* pp = data1d(prio);
    if (idx.shape(0) != prio.shape(0)) throw std::invalid_argument("length mismatch");
    for (py::ssize_t i = 0; i < idx.shape(0); ++i) {
      double v = std::pow(pp[i], alpha_);
      sum_->set(pi[i], v);
      min_->set(pi[i], v);
      max_priority_ = std::max(max_priority_, pp[i]);
    }
  }

  // update_priorities (memory.py:300-320): sequential, so duplicates are last-write-wins.
  void update_priorities(py::array_t<int64_t, py::array::c_style | py::array::forcecast> idx,
                         py::array_t<double, py::array::c_style | py::array::forcecast> prio,
                         int64_t length) {
    const int64_t* pi = data1d(idx);
    const double* pp = data1d(prio);
    if (idx.shape(0) != prio.shape(0)) throw std::invalid_argument("length mismatch");
    for (py::ssize_t i = 0; i < idx.shape(0); ++i) {
      if (!(pp[i] > 0)) throw std::invalid_argument("priority must be > 0");
      if (pi[i] < 0 || pi[i] >= length) throw std::out_of_range("index out of range");
      double v = std::pow(pp[i], alpha_);
      sum_->set(pi[i], v);
      min_->set(pi[i], v);
      max_priority_ = std::max(max_priority_, pp[i]);
    }
  }

  // Stratified proportional sampling (memory.py:242-250). `uniforms` are the B draws of
  // random.random() so the host RNG stream stays identical to the reference's.
  // exclude_last=true reproduces the exclusive-end mass quirk.
  py::array_t<int64_t> sample_proportional(
      py::array_t<double, py::array::c_style | py::array::forcecast> uniforms, int64_t length,
      bool exclude_last) {
    const double* u = data1d(uniforms);
    const int64_t B = uniforms.shape(0);
    double p_total = exclude_last ? sum_->reduce(0, py::int_(length - 1))
                                  : sum_->reduce(0, py::int_(length));
    double every = p_total / static_cast<double>(B);
    py::array_t<int64_t> out(B);
    auto o = out.mutable_unchecked<1>();
    for (int64_t i = 0; i < B; ++i) {
      double mass = u[i] * every + static_cast<double>(i) * every;
      o(i) = sum_->find_prefixsum_idx(mass);
    }
    return out;
  }

  // IS weights (memory.py:284-298): w_i = (p_i N)^-beta / (p_min N)^-beta.
  py::array_t<double> weights(py::array_t<int64_t, py::array::c_style | py::array::forcecast> idx,
                              int64_t length, double beta) {
    if (!(beta > 0)) throw std::invalid_argument("beta must be > 0");
    const int64_t* pi = data1d(idx);
    const double total = sum_->reduce(0, py::none());
    const double p_min = min_->reduce(0, py::none()) / total;
    const double n = static_cast<double>(length);
    const double max_w = std::pow(p_min * n, -beta);
    py::array_t<double> out(idx.shape(0));
    auto o = out.mutable_unchecked<1>();
    for (py::ssize_t i = 0; i < idx.shape(0); ++i) {
      double p_sample = sum_->get(pi[i]) / total;
      double w = std::pow(p_sample * n, -beta);
      o(i) = w / max_w;
    }
    return out;
  }

  Tree& sum_tree() { return *sum_; }
  Tree& min_tree() { return *min_; }
  double max_priority() const { return max_priority_; }
  void set_max_priority(double v) { max_priority_ = v; }
  double alpha() const { return alpha_; }

 private:
  double alpha_;
  double max_priority_;
  std::unique_ptr<Tree> sum_;
  std::unique_ptr<Tree> min_;
};

py::array_t<double> tree_values(const Tree& t) {
  const auto& v = t.values();
  py::array_t<double> out(static_cast<py::ssize_t>(v.size()));
  std::copy(v.begin(), v.end(), out.mutable_data());
  return out;
}

// Batched set for plain trees (sequential => last-write-wins on duplicates).
void tree_set_batch(Tree& t, py::array_t<int64_t, py::array::c_style | py::array::forcecast> idx,
                    py::array_t<double, py::array::c_style | py::array::forcecast> vals) {
  const int64_t* pi = data1d(idx);
  const double* pv = data1d(vals);
  if (idx.shape(0) != vals.shape(0)) throw std::invalid_argument("length mismatch");
  for (py::ssize_t i = 0; i < idx.shape(0); ++i) t.set(pi[i], pv[i]);
}

py::array_t<int64_t> tree_find_batch(const Tree& t,
                                     py::array_t<double, py::array::c_style | py::array::forcecast> m) {
  const double* pm = data1d(m);
  py::array_t<int64_t> out(m.shape(0));
  auto o = out.mutable_unchecked<1>();
  for (py::ssize_t i = 0; i < m.shape(0); ++i) o(i) = t.find_prefixsum_idx(pm[i]);
  return out;
}

// n-step discounted return sum_i gamma^i r_i (memory.py:471-475), vectorised over rows.
py::array_t<double> multi_step_returns(
    py::array_t<double, py::array::c_style | py::array::forcecast> rewards, double gamma) {
  if (rewards.ndim() != 2) throw std::invalid_argument("rewards must be [N, n]");
  const auto r = rewards.unchecked<2>();
  py::array_t<double> out(rewards.shape(0));
  auto o = out.mutable_unchecked<1>();
  for (py::ssize_t i = 0; i < rewards.shape(0); ++i) {
    double ret = 0.0, g = 1.0;
    for (py::ssize_t j = 0; j < rewards.shape(1); ++j) {
      ret += r(i, j) * g;
      g *= gamma;
    }
    o(i) = ret;
  }
  return out;
}

}  // namespace

PYBIND11_MODULE(_apex_cpu, m) {
  m.doc() = "apex_amd native host replay core (segment trees, PER batch ops)";

  py::class_<Tree>(m, "Tree")
      .def(py::init([](int64_t cap, const std::string& op) {
             if (op == "sum") return std::make_unique<Tree>(cap, TreeOp::Sum);
             if (op == "min") return std::make_unique<Tree>(cap, TreeOp::Min);
             throw std::invalid_argument("op must be 'sum' or 'min'");
           }),
           py::arg("capacity"), py::arg("op"))
      .def("set", &Tree::set)
      .def("get", &Tree::get)
      .def("reduce", &Tree::reduce, py::arg("start") = 0, py::arg("end") = py::none())
      .def("find_prefixsum_idx", &Tree::find_prefixsum_idx)
      .def("set_batch", &tree_set_batch)
      .def("find_prefixsum_idx_batch", &tree_find_batch)
      .def("values", &tree_values)
      .def_property_readonly("capacity", &Tree::capacity)
      .def_property_readonly("root", &Tree::root);

  py::class_<PERCore>(m, "PERCore")
      .def(py::init<int64_t, double>(), py::arg("size"), py::arg("alpha"))
      .def("add_max", &PERCore::add_max)
      .def("add_with_priority", &PERCore::add_with_priority)
      .def("update_priorities", &PERCore::update_priorities)
      .def("sample_proportional", &PERCore::sample_proportional, py::arg("uniforms"),
           py::arg("length"), py::arg("exclude_last") = true)
      .def("weights", &PERCore::weights)
      .def("sum_tree", &PERCore::sum_tree, py::return_value_policy::reference_internal)
      .def("min_tree", &PERCore::min_tree, py::return_value_policy::reference_internal)
      .def_property("max_priority", &PERCore::max_priority, &PERCore::set_max_priority)
      .def_property_readonly("alpha", &PERCore::alpha);

  m.def("multi_step_returns", &multi_step_returns);
}
