// wgrad table probe w8c: the library table with block 5 back at 4 waves (CIB 16, COB 128, 3 workgroups per CU, no prefetch).
template <> struct WgCfg<0> { static constexpr int CIB = 32, COB = 128, WCO = 4, WCI = 1, RTILES = 2, MINWG = 512, U = 4, MINB = 2, WAVES = 4; static constexpr bool PF = false, PFA = false; };  // im2col kk=32
template <> struct WgCfg<1> { static constexpr int CIB = 32, COB = 192, WCO = 4, WCI = 2, RTILES = 8, MINWG = 256, U = 8, MINB = 1, WAVES = 8; static constexpr bool PF = true, PFA = true; };
template <> struct WgCfg<2> { static constexpr int CIB = 64, COB = 224, WCO = 2, WCI = 4, RTILES = 8, MINWG = 256, U = 8, MINB = 1, WAVES = 8; static constexpr bool PF = true, PFA = true; };
template <> struct WgCfg<3> { static constexpr int CIB = 32, COB = 96, WCO = 2, WCI = 2, RTILES = 16, MINWG = 512, U = 8, MINB = 2, WAVES = 4; static constexpr bool PF = true, PFA = true; };
template <> struct WgCfg<4> { static constexpr int CIB = 16, COB = 128, WCO = 4, WCI = 1, RTILES = 16, MINWG = 768, U = 8, MINB = 3, WAVES = 4; static constexpr bool PF = false, PFA = false; };
template <> struct WgCfg<5> { static constexpr int CIB = 64, COB = 96, WCO = 2, WCI = 4, RTILES = 16, MINWG = 256, U = 4, MINB = 1, WAVES = 8; static constexpr bool PF = true, PFA = true; };
