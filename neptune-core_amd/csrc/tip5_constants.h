// Tip5 constants (twenty-first 1.0.0 `tip5` module; crate pinned at /root/reference/Cargo.lock:4297).
// Values are data, checked by tests/test_constants.py against the BLAKE3 derivation
// raw_i = u128::from_le_bytes(BLAKE3("Tip5" || i)[..16]) mod p and against the reference KATs.
#pragma once
#include <stdint.h>
namespace nhip {
// Round constants as RAW Montgomery values (x * 2^64 mod p), round-major [round*16 + i].
static constexpr uint64_t TIP5_RC_RAW[80] = {
    0x61ab60dce12a6137ull, 0xd9547ed03c2d8f14ull, 0xa1de063dce16c34aull, 0x876c86765d4cf10bull,
    0x889cfb95a3fe2af2ull, 0x43699f00e0086636ull, 0x7190db575712e44bull, 0xd2b0d4b005bceb49ull,
    0xd483cd36b29f2156ull, 0x44882a5588310f48ull, 0x9f498aa3b091da34ull, 0x79338d4bf1ff20f5ull,
    0x52c5b216fc597178ull, 0x48adad93be758d99ull, 0xfec868b59853d114ull, 0xfb6b0d8a2cc48735ull,
    0x20ef0328ebc0eeecull, 0x5bba58025bdfe8e6ull, 0x27287a2602df87a9ull, 0x4e1934110c7397faull,
    0xa977eae0cf6133cbull, 0x63fc191a6bef3d61ull, 0xaf39b21096b1f98dull, 0x5933202ea3216fc1ull,
    0xbfcf71e4029fd62dull, 0xcc520bfbfb4ad152ull, 0xf774f673e0c840b1ull, 0x0309bc69ad2abfa1ull,
    0x275f3cb27a336665ull, 0x2c8f905ae6ad794bull, 0x61e609b31a9aa328ull, 0x5c92c93af0bb400bull,
    0x56411dbfe9bc674aull, 0x5fc2a26b895bd10cull, 0x3d9f2bf239dfe4f5ull, 0x5ca88c43f0c467e0ull,
    0x2e1c155235b5227bull, 0x3220a672e82efaddull, 0x4b861c4d0fdd1d04ull, 0xeb86ebd60308861full,
    0xbc3902de832913f5ull, 0x516bcbc01bf8f7c6ull, 0x738f27cfac69f270ull, 0xeac8ea36e798f708ull,
    0x4bf937c4aa81ef62ull, 0x220e67469498717dull, 0x07e796f8f9fad5c4ull, 0xf2f6dd71e16d8ff5ull,
    0x7d6e3a407aefd019ull, 0xe73743d7d4c162e9ull, 0xef802e57717a8a87ull, 0x336e6aa553bcde49ull,
    0xf3c8b2265e71152aull, 0x6afb2112f02e0b04ull, 0x255319673d64ddb1ull, 0x3866d0ee91012a32ull,
    0xd22150224702d633ull, 0x12ee85b15e3f4dacull, 0xfcd23eb4c9b208c8ull, 0xd727752f3d490349ull,
    0xaff543b3b670e77eull, 0x17f192d4f48bc718ull, 0xb026adc00615dfdfull, 0xe35c1017dcab5e5bull,
    0x6080bd0671014a42ull, 0x0b8a28b7fe9a2b22ull, 0xae9da4cacc26240dull, 0xd9e5a26b732867a0ull,
    0x2d33784692fe65b8ull, 0xb7eee345dcb6de4cull, 0x59dde50c8f0c9826ull, 0x5ee62a88e059226dull,
    0xf6a203d0a302d668ull, 0x3b6ae69e93fb6a88ull, 0x2be69c3753fb6dbfull, 0xdfff43cb9f9a0f27ull,
    0x5f4fdc6a15b64f4bull, 0x97c0d760903d0ed1ull, 0x14148ebadb21a28bull, 0xf2f24472b971e6c9ull,
};
// S-box lookup table L(x) = (x+1)^3 - 1 mod 257, applied bytewise to raw Montgomery words.
static constexpr uint8_t TIP5_LUT[256] = {
    0, 7, 26, 63, 124, 215, 85, 254, 214, 228, 45, 185, 140, 173, 33, 240,
    29, 177, 176, 32, 8, 110, 87, 202, 204, 99, 150, 106, 230, 14, 235, 128,
    213, 239, 212, 138, 23, 130, 208, 6, 44, 71, 93, 116, 146, 189, 251, 81,
    199, 97, 38, 28, 73, 179, 95, 84, 152, 48, 35, 119, 49, 88, 242, 3,
    148, 169, 72, 120, 62, 161, 166, 83, 175, 191, 137, 19, 100, 129, 112, 55,
    221, 102, 218, 61, 151, 237, 68, 164, 17, 147, 46, 234, 203, 216, 22, 141,
    65, 57, 123, 12, 244, 54, 219, 231, 96, 77, 180, 154, 5, 253, 133, 165,
    98, 195, 205, 134, 245, 30, 9, 188, 59, 142, 186, 197, 181, 144, 92, 31,
    224, 163, 111, 74, 58, 69, 113, 196, 67, 246, 225, 10, 121, 50, 60, 157,
    90, 122, 2, 250, 101, 75, 178, 159, 24, 36, 201, 11, 243, 132, 198, 190,
    114, 233, 39, 52, 21, 209, 108, 238, 91, 187, 18, 104, 194, 37, 153, 34,
    200, 143, 126, 155, 236, 118, 64, 80, 172, 89, 94, 193, 135, 183, 86, 107,
    252, 13, 167, 206, 136, 220, 207, 103, 171, 160, 76, 182, 227, 217, 158, 56,
    174, 4, 66, 109, 139, 162, 184, 211, 249, 47, 125, 232, 117, 43, 16, 42,
    127, 20, 241, 25, 149, 105, 156, 51, 53, 168, 145, 247, 223, 79, 78, 226,
    15, 222, 82, 115, 70, 210, 27, 41, 1, 170, 40, 131, 192, 229, 248, 255,
};
// First column of the circulant MDS matrix: out[i] = sum_j MDS[(i - j) & 15] * in[j].
static constexpr uint32_t TIP5_MDS[16] = {61402, 1108, 28750, 33823, 7454, 43244, 53865, 12034, 56951, 27521, 41351, 40901, 12021, 59689, 26798, 17845};
}  // namespace nhip
