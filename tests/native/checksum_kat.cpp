// The reference's checksum KATs (test/unit/TestChecksum.cpp:46-140, fixtures
// test/data/checksum{1,2}.in, copied verbatim to tests/golden/) run through
// integration/GpuCrc32c.h — a Hdfs::Internal::Checksum subclass compiled against the
// reference's own src/common/Checksum.h — exactly as TEST_F(TestChecksum, SWCrc32c) drives
// its engine: value 0 after construction/reset, every case at 8 alignments, and the
// streamed total of checksum2.in. Built and run by tests/test_reference_headers.py.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <locale>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "GpuCrc32c.h"

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    std::vector<std::pair<uint32_t, std::string>> cases;
    std::vector<std::string> strs;
    uint32_t result = 0;
    {
        std::ifstream in(argv[1]);
        std::string line, s;
        uint32_t v;
        while (std::getline(in, line)) {
            std::stringstream ss(line);
            ss.imbue(std::locale::classic());
            ss >> v >> s;
            cases.emplace_back(v, s);
        }
    }
    {
        std::ifstream in(argv[2]);
        in >> result;
        std::string s;
        while (std::getline(in, s)) strs.push_back(s);
    }
    std::unique_ptr<Hdfs::Internal::Checksum> cs(new Hdfs::Internal::GpuCrc32c());  // through the ABC
    int fails = 0;
    if (cs->getValue() != 0u) ++fails;
    for (const auto &c : cases) {
        const size_t len = c.second.size();
        std::vector<char> buffer(sizeof(uint64_t) + len);
        for (size_t j = 0; j < sizeof(uint64_t); ++j) {
            std::memcpy(&buffer[j], c.second.data(), len);
            cs->reset();
            cs->update(&buffer[j], int(len));
            if (cs->getValue() != c.first) ++fails;
        }
    }
    cs->reset();
    if (cs->getValue() != 0u) ++fails;
    for (auto &s : strs) cs->update(s.data(), int(s.size()));
    if (cs->getValue() != result) ++fails;
    std::printf("cases %zu streamed %zu total %u want %u fails %d\n", cases.size(), strs.size(), cs->getValue(), result,
                fails);
    return fails == 0 && cases.size() == 512 ? 0 : 1;
}
