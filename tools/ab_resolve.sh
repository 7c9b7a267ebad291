# Isolated resolve kernel stats (tools/resolve_w.py) for abtmp/old.so vs abtmp/new.so.
set -eu
for v in old new; do
  cp abtmp/$v.so rogtk_amd/librogtk_hip.so
  echo "#### $v"
  bash tools/profile_resolve_w.sh
done
