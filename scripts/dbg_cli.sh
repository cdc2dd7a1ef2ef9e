cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT/deflate-library-java_amd/python
python3 -c "open('/tmp/z.bin','wb').write(bytes(1<<20))"
timeout -k 5 120 python3 -m ndfl.gzip /tmp/z.bin /tmp/z.gz; echo rc=$?
NDFL_DEBUG=1 timeout -k 5 120 python3 -m ndfl.gunzip /tmp/z.gz /tmp/z.out; echo rc=$?
NDFL_HOST_LINK=1 timeout -k 5 120 python3 -m ndfl.gunzip /tmp/z.gz /tmp/z2.out; echo hostlink rc=$?
