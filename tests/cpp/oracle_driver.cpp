// Drives the CPU oracle (oracle/gi_oracle.cpp, test infrastructure) over scene files in Mode R and
// Mode X, for the sanitizer build in tests/test_host_math.py.
#include <cstdio>
#include <cstdint>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>
extern "C" int gio_render(const char* scn, int w, int h, int mode, int spp, int depth, uint64_t seed, int x0, int y0,
                          int x1, int y1, int threads, double* rgb, int32_t* hit, int32_t* uv, int32_t* ncand,
                          int32_t* nnode, uint8_t* q);
extern "C" const char* gio_last_error(void);
int main(int argc, char** argv) {
    for (int a = 1; a < argc; ++a) {
        std::ifstream f(argv[a]); std::stringstream ss; ss << f.rdbuf(); std::string s = ss.str();
        const int w = 48, h = 40, n = w * h;
        std::vector<double> rgb(n * 3); std::vector<int32_t> hit(n), uv(n * 2), nc(n), nn(n); std::vector<uint8_t> q(n * 3);
        for (int mode = 0; mode < 2; ++mode) {
            int rc = gio_render(s.c_str(), w, h, mode, mode ? 3 : 1, mode ? 5 : 1, 7, 0, 0, w, h, 1, rgb.data(), hit.data(),
                                uv.data(), nc.data(), nn.data(), q.data());
            std::printf("%s mode %d rc %d %s\n", argv[a], mode, rc, rc ? gio_last_error() : "");
        }
    }
    return 0;
}
