# no source change (variants that differ only by -D defines)
PATCHES = []
