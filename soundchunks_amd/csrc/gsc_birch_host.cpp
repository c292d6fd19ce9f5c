// The -py reducer: TFrame.Reduce with PythonReduce set
// (encoder.lpr:837-841) writes the frame's dataset as text and runs
// encoder/cluster.py (extern.pas:350-437), which fits
//     sklearn.cluster.Birch(n_clusters = K, threshold = 0.001, branching_factor = 50)
// and returns Birch.labels_ (only the labels reach the encoder: cluster.py's
// .cluster_centres are replaced by the cluster means of a5).  Restated here
// natively, after the sklearn 1.7.2 / scipy 1.15 code the reference runs:
//   1. the text round trip (extern.pas:363-369, cluster.py:13): every Single
//      is printed by FloatToStr and read back by numpy.loadtxt as a double.
//      FloatToStr(Single) in encoder.exe (@0x100034390 -> @0x100034340)
//      widens to Double and calls FloatToStrFIntl(ffGeneral, Precision 15,
//      Digits 0, fvSingle) (@0x100032a10), whose fvSingle branch
//      (@0x100032b5c) is Str(Single(v):21) with real type single; str_real
//      (@0x10000c240) caps the digits at its per-type table entry
//      (.data 0x10004b950: single -> 10 digits, 2 exponent digits), so the
//      text carries 10 significant digits: v -> strtod("%.9e" of v);
//   2. the CF tree (sklearn/cluster/_birch.py: _CFNode.insert_cf_subcluster,
//      _CFSubcluster.update / merge_subcluster, _split_node), in sample order;
//   3. the global step AgglomerativeClustering(n_clusters = K) = Ward linkage
//      of the leaf subcluster centroids (scipy.cluster.hierarchy.ward:
//      euclidean pdist, nearest-neighbour chain, Lance-Williams Ward update,
//      stable sort by height, union-find relabelling) cut by sklearn's _hc_cut
//      (a max-heap of node ids, labels in heap order);
//   4. labels_ = the global label of each sample's nearest subcluster centroid
//      (Birch._predict -> sklearn ArgKmin: max(0, (|x|^2 + (-2 x.c)) + |c|^2),
//      first minimum).
// Numerics: every dot product, norm and product matrix follows the summation
// order of the BLAS / einsum call numpy and scipy make for it (gsc_npblas.h:
// np.dot of two vectors and scipy's _dot -> OpenBLAS ddot; np.dot(M, v) ->
// dgemv_t; euclidean_distances in _split_node -> einsum row norms and dsyrk;
// the predict middle term -> dgemm); pdist is a sequential sum (scipy's).
// Labels equal cluster.py's on every committed fixture
// (tests/golden/birch_*.npz, tools: tests/golden/make_birch.py).
// The O(m^2) Ward step and the O(N m) predict run on the device
// (gsc_birch.hip); the CF tree is sequential by construction and runs here.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gsc_npblas.h"

namespace gsc {

extern "C" int gsc_ward_linkage_dev(int m, int d, const double* centers, double* Z);
extern "C" int gsc_birch_predict_dev(int n, int d, const double* X, int m, const double* centers, int* argmin);

namespace {

constexpr double kThreshold = 0.001;
constexpr int kBranching = 50;

// np.dot of two vectors (OpenBLAS ddot order)
double dotv(const double* a, const double* b, int d) { return npblas::np_ddot(a, b, d); }

struct Sub {
    int n = 0;
    std::vector<double> ls;  // linear sum (empty: the int 0 of a fresh _CFSubcluster)
    double ss = 0.0;         // squared sum
    std::vector<double> centroid;
    double sqn = 0.0;        // |centroid|^2
    int child = -1;          // node index
};

struct Node {
    bool leaf = true;
    std::vector<int> subs;             // subcluster indices
    std::vector<double> cent, sqn;     // init_centroids_ / init_sq_norm_ rows (branching_factor + 1)
    int prev = -1, next = -1;          // leaf chain
};

class Birch {
   public:
    Birch(int d) : d_(d) {}

    int new_node(bool leaf) {
        Node nd;
        nd.leaf = leaf;
        nd.cent.assign(size_t(kBranching + 1) * d_, 0.0);
        nd.sqn.assign(size_t(kBranching + 1), 0.0);
        nodes_.push_back(std::move(nd));
        return int(nodes_.size()) - 1;
    }
    int new_sub() {
        subs_.emplace_back();
        return int(subs_.size()) - 1;
    }

    void append(int node, int s) {
        Node& nd = nodes_[node];
        const size_t k = nd.subs.size();
        nd.subs.push_back(s);
        std::memcpy(&nd.cent[k * d_], subs_[s].centroid.data(), sizeof(double) * d_);
        nd.sqn[k] = subs_[s].sqn;
    }

    // _CFSubcluster.update
    void update(int self, int other) {
        Sub& a = subs_[self];
        const Sub& b = subs_[other];
        a.n += b.n;
        if (a.ls.empty()) a.ls.assign(size_t(d_), 0.0);
        for (int k = 0; k < d_; ++k) a.ls[k] = a.ls[k] + b.ls[k];
        a.ss = a.ss + b.ss;
        a.centroid.resize(size_t(d_));
        for (int k = 0; k < d_; ++k) a.centroid[k] = a.ls[k] / double(a.n);
        a.sqn = dotv(a.centroid.data(), a.centroid.data(), d_);
    }

    // _CFSubcluster.merge_subcluster
    bool merge(int self, int nom) {
        Sub& a = subs_[self];
        const Sub& b = subs_[nom];
        const double new_ss = a.ss + b.ss;
        std::vector<double> new_ls(static_cast<size_t>(d_));
        for (int k = 0; k < d_; ++k) new_ls[k] = a.ls[k] + b.ls[k];
        const int new_n = a.n + b.n;
        const double inv = 1.0 / double(new_n);
        std::vector<double> c(static_cast<size_t>(d_));
        for (int k = 0; k < d_; ++k) c[k] = inv * new_ls[k];
        const double new_sqn = dotv(c.data(), c.data(), d_);
        const double sq_radius = new_ss / double(new_n) - new_sqn;
        if (sq_radius <= kThreshold * kThreshold) {
            a.n = new_n;
            a.ls.swap(new_ls);
            a.ss = new_ss;
            a.centroid.swap(c);
            a.sqn = new_sqn;
            return true;
        }
        return false;
    }

    // _split_node: farthest pair by euclidean_distances(centroids, squared=True)
    std::pair<int, int> split(int node) {
        const int s1 = new_sub(), s2 = new_sub();
        const bool leaf = nodes_[node].leaf;
        const int n1 = new_node(leaf), n2 = new_node(leaf);
        subs_[s1].child = n1;
        subs_[s2].child = n2;
        if (leaf) {
            const int prev = nodes_[node].prev, next = nodes_[node].next;
            if (prev >= 0) nodes_[prev].next = n1;
            nodes_[n1].prev = prev;
            nodes_[n1].next = n2;
            nodes_[n2].prev = n1;
            nodes_[n2].next = next;
            if (next >= 0) nodes_[next].prev = n2;
        }
        const std::vector<int> members = nodes_[node].subs;  // copy: the node is dropped
        const int m = int(members.size());
        const double* C = nodes_[node].cent.data();
        // euclidean_distances(centroids_, squared=True) with Y = X: the passed
        // Y_norm_squared is unused (Y is X); XX = row_norms (einsum), then
        // -2 * (X @ X.T) (dsyrk) + XX[i] + XX[j], clipped at 0, zero diagonal
        if (m != kBranching + 1) std::abort();  // _split_node only ever sees branching_factor + 1 rows
        std::vector<double> xx(static_cast<size_t>(m)), dist(size_t(m) * m);
        for (int i = 0; i < m; ++i) xx[i] = npblas::np_einsum_sq(C + size_t(i) * d_, d_);
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < m; ++j) {
                double v = -2.0 * npblas::np_syrk51(C, d_, i, j);
                v = v + xx[i];
                v = v + xx[j];
                dist[size_t(i) * m + j] = i == j ? 0.0 : (v < 0.0 ? 0.0 : v);  // np.maximum(v, 0)
            }
        size_t far = 0;
        for (size_t k = 1; k < dist.size(); ++k)
            if (dist[k] > dist[far]) far = k;
        const int f1 = int(far / size_t(m)), f2 = int(far % size_t(m));
        for (int idx = 0; idx < m; ++idx) {
            const bool closer1 = idx == f1 || dist[size_t(f1) * m + idx] < dist[size_t(f2) * m + idx];
            const int s = members[idx];
            if (closer1) {
                append(n1, s);
                update(s1, s);
            } else {
                append(n2, s);
                update(s2, s);
            }
        }
        return {s1, s2};
    }

    // _CFNode.insert_cf_subcluster; true = the node must be split
    bool insert(int node, int s) {
        if (nodes_[node].subs.empty()) {
            append(node, s);
            return false;
        }
        const Node& nd = nodes_[node];
        const int m = int(nd.subs.size());
        const double* q = subs_[s].centroid.data();
        int best = 0;
        double bd = 0.0;
        for (int i = 0; i < m; ++i) {
            double v = npblas::np_gemv_row(&nd.cent[size_t(i) * d_], q, d_, m, i);  // np.dot(centroids_, c)
            v = v * -2.0;
            v = v + nd.sqn[i];
            if (i == 0 || v < bd) {
                bd = v;
                best = i;
            }
        }
        const int closest = nd.subs[best];
        if (subs_[closest].child >= 0) {
            const bool split_child = insert(subs_[closest].child, s);
            if (!split_child) {
                update(closest, s);
                std::memcpy(&nodes_[node].cent[size_t(best) * d_], subs_[closest].centroid.data(), sizeof(double) * d_);
                nodes_[node].sqn[best] = subs_[closest].sqn;
                return false;
            }
            const auto ns = split(subs_[closest].child);
            // update_split_subclusters: the first subcluster takes the closest one's place
            Node& n2 = nodes_[node];
            n2.subs[best] = ns.first;
            std::memcpy(&n2.cent[size_t(best) * d_], subs_[ns.first].centroid.data(), sizeof(double) * d_);
            n2.sqn[best] = subs_[ns.first].sqn;
            append(node, ns.second);
            return int(nodes_[node].subs.size()) > kBranching;
        }
        if (merge(closest, s)) {
            std::memcpy(&nodes_[node].cent[size_t(best) * d_], subs_[closest].centroid.data(), sizeof(double) * d_);
            nodes_[node].sqn[best] = subs_[closest].sqn;
            return false;
        }
        append(node, s);
        return int(nodes_[node].subs.size()) > kBranching;
    }

    // Birch._fit: the leaf subcluster centroids in leaf-chain order
    std::vector<double> fit(int n, const double* X) {
        int root = new_node(true);
        const int dummy = new_node(true);
        nodes_[dummy].next = root;
        nodes_[root].prev = dummy;
        for (int i = 0; i < n; ++i) {
            const int s = new_sub();
            Sub& sb = subs_[s];
            sb.n = 1;
            sb.ls.assign(X + size_t(i) * d_, X + size_t(i + 1) * d_);
            sb.centroid = sb.ls;
            sb.ss = sb.sqn = dotv(sb.ls.data(), sb.ls.data(), d_);
            if (insert(root, s)) {
                const auto ns = split(root);
                root = new_node(false);
                append(root, ns.first);
                append(root, ns.second);
            }
        }
        std::vector<double> centers;
        for (int lf = nodes_[dummy].next; lf >= 0; lf = nodes_[lf].next)
            centers.insert(centers.end(), nodes_[lf].cent.begin(),
                           nodes_[lf].cent.begin() + long(nodes_[lf].subs.size() * size_t(d_)));
        return centers;
    }

   private:
    int d_;
    std::vector<Node> nodes_;
    std::vector<Sub> subs_;
};

// scipy's LinkageUnionFind relabelling of the sorted nn-chain merges
void scipy_label(std::vector<double>& Z, int n) {
    std::vector<int> parent(static_cast<size_t>(2 * n - 1));
    for (int i = 0; i < 2 * n - 1; ++i) parent[i] = i;
    std::vector<int> size(size_t(2 * n - 1), 1);
    int next_label = n;
    auto find = [&](int x) {
        int p = x;
        while (parent[x] != x) x = parent[x];
        while (parent[p] != x) {
            const int q = parent[p];
            parent[p] = x;
            p = q;
        }
        return x;
    };
    for (int i = 0; i < n - 1; ++i) {
        const int x = int(Z[size_t(i) * 4]), y = int(Z[size_t(i) * 4 + 1]);
        const int xr = find(x), yr = find(y);
        Z[size_t(i) * 4] = double(std::min(xr, yr));
        Z[size_t(i) * 4 + 1] = double(std::max(xr, yr));
        parent[xr] = next_label;
        parent[yr] = next_label;
        size[next_label] = size[xr] + size[yr];
        Z[size_t(i) * 4 + 3] = double(size[next_label]);
        ++next_label;
    }
}

// sklearn _hc_cut: heapq semantics on negated node ids
void heap_push(std::vector<long>& h, long v) {
    h.push_back(v);
    size_t pos = h.size() - 1;
    while (pos > 0) {  // _siftdown(heap, 0, pos)
        const size_t parent = (pos - 1) >> 1;
        if (v < h[parent]) {
            h[pos] = h[parent];
            pos = parent;
            continue;
        }
        break;
    }
    h[pos] = v;
}
void heap_siftup(std::vector<long>& h, size_t pos) {  // heapq._siftup
    const size_t end = h.size(), start = pos;
    const long item = h[pos];
    size_t child = 2 * pos + 1;
    while (child < end) {
        const size_t right = child + 1;
        if (right < end && !(h[child] < h[right])) child = right;
        h[pos] = h[child];
        pos = child;
        child = 2 * pos + 1;
    }
    h[pos] = item;
    // _siftdown(heap, start, pos)
    const long v = h[pos];
    while (pos > start) {
        const size_t parent = (pos - 1) >> 1;
        if (v < h[parent]) {
            h[pos] = h[parent];
            pos = parent;
            continue;
        }
        break;
    }
    h[pos] = v;
}
long heap_pushpop(std::vector<long>& h, long v) {
    if (!h.empty() && h[0] < v) {
        std::swap(v, h[0]);
        heap_siftup(h, 0);
    }
    return v;
}

std::vector<int> hc_cut(int K, const std::vector<int>& children, int n_leaves) {
    std::vector<long> nodes{-(long(std::max(children[children.size() - 2], children[children.size() - 1])) + 1)};
    for (int it = 0; it < K - 1; ++it) {
        const long top = -nodes[0] - n_leaves;
        const long c0 = children[size_t(top) * 2], c1 = children[size_t(top) * 2 + 1];
        heap_push(nodes, -c0);
        heap_pushpop(nodes, -c1);
    }
    std::vector<int> label(size_t(n_leaves), 0);
    std::vector<long> stack;
    for (size_t i = 0; i < nodes.size(); ++i) {
        stack.assign(1, -nodes[i]);
        while (!stack.empty()) {  // _hc_get_descendent
            const long x = stack.back();
            stack.pop_back();
            if (x < n_leaves) {
                label[size_t(x)] = int(i);
            } else {
                stack.push_back(children[size_t(x - n_leaves) * 2]);
                stack.push_back(children[size_t(x - n_leaves) * 2 + 1]);
            }
        }
    }
    return label;
}

}  // namespace

// labels of N samples (N x d Single) reduced to K clusters; 0 or an error
int birch_reduce_labels(int n, int d, const float* feat, int K, int* labels, std::string* err) {
    // FloatToStr -> numpy.loadtxt round trip (extern.pas:363-369, cluster.py:13):
    // 10 significant digits (FloatToStr(Single), see the header)
    std::vector<double> X(size_t(n) * d);
    char buf[64];
    for (size_t k = 0; k < X.size(); ++k) {
        std::snprintf(buf, sizeof(buf), "%.9e", double(feat[k]));
        X[k] = std::strtod(buf, nullptr);
    }
    Birch b(d);
    const std::vector<double> centers = b.fit(n, X.data());
    const int m = int(centers.size() / size_t(d));
    std::vector<int> sub_label(static_cast<size_t>(m));
    if (m < K) {  // not enough subclusters: subcluster_labels_ = arange (sklearn warns)
        for (int i = 0; i < m; ++i) sub_label[i] = i;
    } else {
        std::vector<double> Z(size_t(m > 1 ? m - 1 : 1) * 4);
        if (m > 1) {
            const int wr = gsc_ward_linkage_dev(m, d, centers.data(), Z.data());
            if (wr == -2) {
                char msg[160];
                std::snprintf(msg, sizeof(msg),
                              "Birch: Ward linkage of %d subclusters needs %.1f GB of device memory for its "
                              "condensed distance matrix, more than is free",
                              m, double(m) * double(m - 1) / 2.0 * 8.0 / 1e9);
                *err = msg;
                return -1;
            }
            if (wr != 0) {
                *err = "Birch: Ward linkage on the device failed";
                return -1;
            }
            // sort by height (numpy mergesort: stable), then relabel
            std::vector<int> order(static_cast<size_t>(m - 1));
            for (int i = 0; i < m - 1; ++i) order[i] = i;
            std::stable_sort(order.begin(), order.end(),
                             [&](int a, int c) { return Z[size_t(a) * 4 + 2] < Z[size_t(c) * 4 + 2]; });
            std::vector<double> Zs(Z.size());
            for (int i = 0; i < m - 1; ++i) std::memcpy(&Zs[size_t(i) * 4], &Z[size_t(order[i]) * 4], 4 * sizeof(double));
            scipy_label(Zs, m);
            std::vector<int> children(size_t(m - 1) * 2);
            for (int i = 0; i < m - 1; ++i) {
                children[size_t(i) * 2] = int(Zs[size_t(i) * 4]);
                children[size_t(i) * 2 + 1] = int(Zs[size_t(i) * 4 + 1]);
            }
            sub_label = hc_cut(K, children, m);
        } else {
            sub_label[0] = 0;
        }
    }
    std::vector<int> am(static_cast<size_t>(n));
    if (gsc_birch_predict_dev(n, d, X.data(), m, centers.data(), am.data()) != 0) {
        *err = "Birch: predict on the device failed";
        return -1;
    }
    for (int i = 0; i < n; ++i) labels[i] = sub_label[size_t(am[i])];
    return 0;
}

}  // namespace gsc
