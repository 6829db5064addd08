# round-4 closing counters after the LDS stride change (profile.sh: kernel
# trace + PMC passes of the bench command)
set -u
bash scripts/profile.sh r04b || exit 1
