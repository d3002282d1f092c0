// wgrad table probe: blocks 2, 3, 5, 6 as one 8-wave workgroup per CU (output block over 8 waves, 64-channel
// ci blocks where the waves need them) with the next tile's dZ / A rows prefetched into registers.
template <> struct WgCfg<0> { static constexpr int CIB = 32, COB = 128, WCO = 4, WCI = 1, RTILES = 2, MINWG = 512, U = 4, MINB = 2, WAVES = 4; static constexpr bool PF = false, PFA = false; };
template <> struct WgCfg<1> { static constexpr int CIB = 32, COB = 192, WCO = 4, WCI = 2, RTILES = 8, MINWG = 256, U = 8, MINB = 1, WAVES = 8; static constexpr bool PF = true, PFA = true; };
template <> struct WgCfg<2> { static constexpr int CIB = 64, COB = 224, WCO = 2, WCI = 4, RTILES = 8, MINWG = 256, U = 8, MINB = 1, WAVES = 8; static constexpr bool PF = true, PFA = true; };
template <> struct WgCfg<3> { static constexpr int CIB = 32, COB = 96, WCO = 2, WCI = 2, RTILES = 16, MINWG = 512, U = 8, MINB = 2, WAVES = 4; static constexpr bool PF = true, PFA = true; };
template <> struct WgCfg<4> { static constexpr int CIB = 32, COB = 128, WCO = 4, WCI = 2, RTILES = 16, MINWG = 256, U = 8, MINB = 1, WAVES = 8; static constexpr bool PF = true, PFA = true; };
template <> struct WgCfg<5> { static constexpr int CIB = 64, COB = 96, WCO = 2, WCI = 4, RTILES = 16, MINWG = 256, U = 4, MINB = 1, WAVES = 8; static constexpr bool PF = true, PFA = true; };
