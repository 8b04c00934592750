source tools/gpu_steps.sh
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
