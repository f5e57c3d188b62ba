set -e
for r in 1 2; do bash tools/ab_args.sh "--groups 3" "--groups 4" "--groups 6"; done
