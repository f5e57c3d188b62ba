# timing variant: planned rows without their literal footers (wrong outputs)
PATCHES = [("backend_hip.hip", "store_literal(p16, rdst, rn, row_lit_len(w1.x), w2.z, w2.w, 16);", "(void)0;")]
