// oracle/ref_cuda_ls.cpp — TEST INFRASTRUCTURE ONLY.
//
// Trace driver for the reference's CUDA-path line searches: linked with the reference's own
// parallel-implementation/line_search.cpp, vector_utils.cpp and functions.cpp, compiled where
// they lie under /root/reference (oracle/Makefile target `ref`), never copied. It runs one of
// the four searches (line_search.h:18-47) from x along d with the gradient g on the reference's
// rosenbrock (functions.cpp:25-48) and records what the oracle's restatement
// (orc_cuda_line_search) must reproduce: the returned step and every f / grad call.
//
//   ref_cuda_ls <method> <in.bin> <out_prefix>
//     in.bin   : int64 n, then x, d, g (n doubles each)
//     out      : <prefix>.alpha.bin (1 double), <prefix>.f.bin (every f() value, in call order),
//                <prefix>.g.bin (per grad() call: checksum c1, c2 of its argument, |grad|
//                left to right as uint64 bits)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include <line_search.h>  // parallel-implementation/line_search.h:14-47

using std::vector;

double rosenbrock(const vector<double>& X);           // functions.cpp:25-35
vector<double> rosenbrock_grad(const vector<double>& X);  // functions.cpp:37-48

static vector<double> g_f;
static vector<uint64_t> g_g;

static void checksum(const vector<double>& x, uint64_t* c1, uint64_t* c2) {
    uint64_t a = 0, b = 0;
    for (size_t i = 0; i < x.size(); ++i) {
        uint64_t u;
        std::memcpy(&u, &x[i], 8);
        a += u;
        b += (uint64_t)(i + 1) * u;
    }
    *c1 = a;
    *c2 = b;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s <backtracking|interpolation|wolfe|backtracking_wolfe> <in.bin> <prefix>\n",
                     argv[0]);
        return 2;
    }
    const std::string method = argv[1];
    FILE* fp = std::fopen(argv[2], "rb");
    if (!fp) return 2;
    int64_t n = 0;
    if (std::fread(&n, 8, 1, fp) != 1 || n < 1) return 2;
    vector<double> x(n), d(n), g(n);
    if (std::fread(x.data(), 8, n, fp) != (size_t)n || std::fread(d.data(), 8, n, fp) != (size_t)n ||
        std::fread(g.data(), 8, n, fp) != (size_t)n)
        return 2;
    std::fclose(fp);
    const std::function<double(vector<double>)> f = [](vector<double> v) {
        const double r = rosenbrock(v);
        g_f.push_back(r);
        return r;
    };
    const std::function<vector<double>(vector<double>)> grad = [](vector<double> v) {
        vector<double> gr = rosenbrock_grad(v);
        uint64_t c1, c2, nb;
        checksum(v, &c1, &c2);
        double s = 0.0;
        for (double e : gr) s += e * e;
        s = __builtin_sqrt(s);
        std::memcpy(&nb, &s, 8);
        g_g.push_back(c1);
        g_g.push_back(c2);
        g_g.push_back(nb);
        return gr;
    };
    double alpha;
    if (method == "backtracking")
        alpha = backtrackingLineSearch(x, d, f, g);
    else if (method == "interpolation")
        alpha = armijoInterpolationLineSearch(x, d, f, g);
    else if (method == "wolfe")
        alpha = wolfeInterpolationLineSearch(x, d, f, grad, g);
    else if (method == "backtracking_wolfe")
        alpha = backtrackingWolfeLineSearch(x, d, f, grad, g);
    else
        return 2;
    const std::string pre = argv[3];
    FILE* fa = std::fopen((pre + ".alpha.bin").c_str(), "wb");
    FILE* ff = std::fopen((pre + ".f.bin").c_str(), "wb");
    FILE* fg = std::fopen((pre + ".g.bin").c_str(), "wb");
    if (!fa || !ff || !fg) return 2;
    std::fwrite(&alpha, 8, 1, fa);
    if (!g_f.empty()) std::fwrite(g_f.data(), 8, g_f.size(), ff);
    if (!g_g.empty()) std::fwrite(g_g.data(), 8, g_g.size(), fg);
    std::fclose(fa);
    std::fclose(ff);
    std::fclose(fg);
    return 0;
}
