# timing variant: planned rows without reading their destination as kept (wrong outputs)
PATCHES = [("backend_hip.hip", "const uint4 cur = live ? load_cur16(p16, rdst, rn, rvalid) : z4;", "const uint4 cur = z4;")]
