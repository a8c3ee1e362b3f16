// ORB vocabulary file parsing (host only; no device needed).
//
// TemplatedVocabulary::loadFromBinaryFile (Thirdparty/DBoW2/DBoW2/
// TemplatedVocabulary.h:1469-1510): header {nb_nodes, size_node, k, L,
// scoring, weighting} (4 x uint32 + 2 x int32), then records of size_node
// bytes {int32 parent, 32 descriptor bytes, float weight, bool is_leaf}. The
// reference reads records while !eof(): the read that hits the end leaves the
// buffer as it was, so the last record is appended a second time (a duplicate
// last child of the same parent, and a duplicate word when it is a leaf).
// The tree is rebuilt exactly that way here; the duplicate never wins a
// descent (it ties with its original, which comes first).
//
// TemplatedVocabulary::loadFromTextFile (:1352-1432): first line "k L
// scoring weighting", then per node "parent is_leaf d0 .. d31 weight". The
// reference turns a trailing empty line into an extra root child with
// uninitialised descriptor bytes; empty lines are skipped here instead.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/gfslam/abi.h"

namespace {

struct Tree {
    int k = 0, L = 0, scoring = 0, weighting = 0;
    std::vector<int32_t> parent;
    std::vector<uint8_t> desc, leaf;
    std::vector<double> weight;
    void root() {
        parent.assign(1, -1);
        desc.assign(32, 0);
        leaf.assign(1, 0);
        weight.assign(1, 0.0);
    }
};

bool ends_with(const std::string& s, const std::string& suf) {
    return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

int read_binary(const char* path, Tree& T) {
    std::ifstream f(path, std::ios::in | std::ios::binary);
    if (!f) return GF_ERR_ARG;
    uint32_t nb_nodes = 0, size_node = 0;
    int32_t hdr[4];
    f.read((char*)&nb_nodes, 4);
    f.read((char*)&size_node, 4);
    f.read((char*)hdr, 16);
    if (!f || size_node < 41 || nb_nodes < 2) return GF_ERR_ARG;
    T.k = hdr[0];
    T.L = hdr[1];
    T.scoring = hdr[2];
    T.weighting = hdr[3];
    T.root();
    std::vector<char> buf(size_node, 0);
    bool any = false;
    while (!f.eof()) {
        f.read(buf.data(), size_node);
        if (!any && f.gcount() == 0) return GF_ERR_ARG;
        any = true;
        int32_t par;
        float w;
        std::memcpy(&par, buf.data(), 4);
        std::memcpy(&w, buf.data() + 36, 4);
        if (par < 0 || par >= (int32_t)T.parent.size()) return GF_ERR_ARG;
        T.parent.push_back(par);
        T.desc.insert(T.desc.end(), buf.begin() + 4, buf.begin() + 36);
        T.weight.push_back((double)w);
        T.leaf.push_back(buf[40] != 0);
    }
    return GF_OK;
}

int read_text(const char* path, Tree& T) {
    std::ifstream f(path);
    if (!f) return GF_ERR_ARG;
    std::string s;
    if (!std::getline(f, s)) return GF_ERR_ARG;
    std::stringstream hs(s);
    int n1 = -1, n2 = -1;
    hs >> T.k >> T.L >> n1 >> n2;
    if (T.k < 0 || T.k > 20 || T.L < 1 || T.L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) return GF_ERR_ARG;
    T.scoring = n1;
    T.weighting = n2;
    T.root();
    while (std::getline(f, s)) {
        if (s.find_first_not_of(" \t\r") == std::string::npos) continue;
        std::stringstream ss(s);
        int pid = 0, is_leaf = 0;
        ss >> pid >> is_leaf;
        if (!ss || pid < 0 || pid >= (int)T.parent.size()) return GF_ERR_ARG;
        uint8_t d[32];
        for (int i = 0; i < 32; i++) {
            int v = 0;
            ss >> v;
            d[i] = (uint8_t)v;
        }
        double w = 0;
        ss >> w;
        T.parent.push_back(pid);
        T.desc.insert(T.desc.end(), d, d + 32);
        T.weight.push_back(w);
        T.leaf.push_back(is_leaf > 0);
    }
    return GF_OK;
}

}  // namespace

extern "C" int gf_vocab_read(const char* path, gf_vocab_arrays* out) {
    if (!path || !out) return GF_ERR_ARG;
    Tree T;
    const int rc = ends_with(path, ".txt") ? read_text(path, T) : read_binary(path, T);
    if (rc) return rc;
    const int n = (int)T.parent.size();
    if (out->parent) {
        if (out->nnodes < n || !out->desc || !out->weight || !out->is_leaf) return GF_ERR_CAP;
        std::memcpy(out->parent, T.parent.data(), 4 * (size_t)n);
        std::memcpy(out->desc, T.desc.data(), 32 * (size_t)n);
        std::memcpy(out->weight, T.weight.data(), 8 * (size_t)n);
        std::memcpy(out->is_leaf, T.leaf.data(), (size_t)n);
    }
    out->k = T.k;
    out->L = T.L;
    out->scoring = T.scoring;
    out->weighting = T.weighting;
    out->nnodes = n;
    return GF_OK;
}

extern "C" int gf_vocab_save_binary(const gf_vocab_arrays* t, const char* path) {
    if (!t || !path || !t->parent || !t->desc || !t->weight || t->nnodes < 1) return GF_ERR_ARG;
    const int n = t->nnodes;
    std::vector<uint8_t> has_child((size_t)n, 0);
    for (int i = 1; i < n; i++) {
        if (t->parent[i] < 0 || t->parent[i] >= n) return GF_ERR_ARG;
        has_child[(size_t)t->parent[i]] = 1;
    }
    std::ofstream f(path, std::ios::out | std::ios::binary);
    if (!f) return GF_ERR_ARG;
    const uint32_t nb_nodes = (uint32_t)n, size_node = 4 + 32 + 4 + 1;
    const int32_t hdr[4] = {t->k, t->L, t->scoring, t->weighting};
    f.write((const char*)&nb_nodes, 4);
    f.write((const char*)&size_node, 4);
    f.write((const char*)hdr, 16);
    for (int i = 1; i < n; i++) {
        const uint32_t par = (uint32_t)t->parent[i];
        const float w = (float)t->weight[i];
        const uint8_t leaf = has_child[(size_t)i] ? 0 : 1;
        f.write((const char*)&par, 4);
        f.write((const char*)t->desc + 32 * (size_t)i, 32);
        f.write((const char*)&w, 4);
        f.write((const char*)&leaf, 1);
    }
    return f ? GF_OK : GF_ERR_ARG;
}
