# Full GPU suite + smoke at HEAD.
bash scripts/steps.sh r05c \
 "pytest|1000|python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'"
