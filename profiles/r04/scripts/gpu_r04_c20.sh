# final-tree counters (default scheduler): kernel trace + PMC passes of the bench command
set -u
bash scripts/profile.sh r04final || exit 1
