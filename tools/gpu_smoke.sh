# smoke() of __graft_entry__ on the GPU box (as the driver runs it)
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
