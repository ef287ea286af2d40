// The assertions of util/crc32c_test.cc:12-53, restated against the drop-in header and linked to
// libkvsep_crc32c.so.  Exit code 0 = all pass.  Built and run by tests/test_cpp_dropin.py.
#include <cstdio>
#include <cstring>

#include "kvsep_leveldb_crc32c.h"

using namespace leveldb::crc32c;

static int failures = 0;
#define EXPECT(c)                                                  \
  do {                                                             \
    if (!(c)) {                                                    \
      std::printf("FAILED line %d: %s\n", __LINE__, #c);           \
      ++failures;                                                  \
    }                                                              \
  } while (0)

int main() {
  char buf[32];
  std::memset(buf, 0, sizeof(buf));
  EXPECT(0x8a9136aa == Value(buf, sizeof(buf)));
  std::memset(buf, 0xff, sizeof(buf));
  EXPECT(0x62a8ab43 == Value(buf, sizeof(buf)));
  for (int i = 0; i < 32; i++) buf[i] = static_cast<char>(i);
  EXPECT(0x46dd794e == Value(buf, sizeof(buf)));
  for (int i = 0; i < 32; i++) buf[i] = static_cast<char>(31 - i);
  EXPECT(0x113fdb5c == Value(buf, sizeof(buf)));
  const unsigned char pdu[48] = {0x01, 0xc0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x14, 0, 0, 0, 0, 0, 0x04, 0,
                                 0, 0, 0, 0x14, 0, 0, 0, 0x18, 0x28, 0, 0, 0, 0, 0, 0, 0, 0x02, 0, 0, 0, 0, 0, 0, 0};
  EXPECT(0xd9963a56 == Value(reinterpret_cast<const char*>(pdu), sizeof(pdu)));
  EXPECT(Value("a", 1) != Value("foo", 3));
  EXPECT(Value("hello world", 11) == Extend(Value("hello ", 6), "world", 5));
  uint32_t crc = Value("foo", 3);
  EXPECT(crc != Mask(crc));
  EXPECT(crc != Mask(Mask(crc)));
  EXPECT(crc == Unmask(Mask(crc)));
  EXPECT(crc == Unmask(Unmask(Mask(Mask(crc)))));
  EXPECT(kvsep_accelerated_crc32c(0, "TestCRCBuffer", 13) == 0xdcbc59fa);  // util/crc32c.cc:267-274
  std::printf("%s\n", failures ? "FAIL" : "PASS");
  return failures ? 1 : 0;
}
