set -e
bash tools/ab_variants.sh oldchunk newchunk oldchunk newchunk oldchunk newchunk
