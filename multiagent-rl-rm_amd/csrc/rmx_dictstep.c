/* rmx_dictstep.c — the per-step host path of rmx.compat.RMEnvironmentWrapper.step in C (CPython C API).
 *
 * The reference's dict API (rm_environment_wrapper.py:43-107) returns five dicts per env step; at N = 1 the Python
 * that turns the engine's output record into those dicts took ~3.3 us of a ~7.9 us step on the GPU box (the rest
 * is the host <-> device mailbox round trip, rmx_step_sync_begin / rmx_sync_wait).  This module runs the same
 * steps without the interpreter loop:
 *   actions dict -> action indices -> rmx_step_sync_begin (the request goes out) -> the previous-state bookkeeping
 *   (overlapping the round trip) -> rmx_sync_wait -> the output record -> agent.set_position, RM labels, the five
 *   dicts, the env's active_agents / agent_fail / agent_steps / timestep mirrors.
 * It calls the reference objects' own methods and attributes exactly where rmx/compat.py does, so a reference
 * object graph sees the same calls, and builds a use_qrm learner's infos["qrm_experience"] tuples
 * (rm_environment_wrapper.py:78-89, 122-183) from the engine's QRM columns.  Anything off the common path returns None
 * and the Python implementation runs instead: a learner that turned use_qrm on since the engine was built without QRM
 * columns (the Python path rebuilds it), an action that is not an object with a known .name, and "wait" under
 * FrozenLake slip (the reference's KeyError path).
 *
 * Built by multiagent-rl-rm_amd/csrc/Makefile (gcc, the interpreter's headers); no HIP, no torch. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

#define MAXA 8 /* RMX_MAX_AGENTS */
#define CTX_ITEMS 20

/* getattr(x, name, default) without building an AttributeError: the public name from CPython 3.13 on */
#if PY_VERSION_HEX >= 0x030D0000
#define LOOKUP_ATTR PyObject_GetOptionalAttr
#else
#define LOOKUP_ATTR _PyObject_LookupAttr
#endif
#ifndef RMX_DICTSTEP_HASH /* the Makefile passes the first 16 hex digits of this file's SHA-256 */
#define RMX_DICTSTEP_HASH "unknown"
#endif

typedef int (*begin_fn)(void* h, const int32_t* actions_host, int autoreset, void* stream);
typedef int (*wait_fn)(void* h, const void* out_host);

/* interned attribute / key names */
static PyObject *s_name, *s_use_qrm, *s_state, *s_current_state, *s_set_position, *s_active_agents, *s_agent_fail,
    *s_agent_steps, *s_timestep, *s_learning_algorithm, *s_position, *k_pos_x, *k_pos_y;
static PyObject *k_prev_s, *k_s, *k_Renv, *k_RQ, *k_prev_q, *k_q, *k_reward_machine, *k_env_terminated,
    *k_rm_terminated, *k_qrm_experience;

/* step(ctx, actions) -> (obs, rewards, terms, truncs, infos) | None (take the Python path) | int rc (a C-ABI error)
 * ctx = (h, begin, wait, act_ptr, bufs_ptr, out_ptr, fl_kind, fl_slip, names, agents, rms, labels, getl, env,
 *        action_index, qrm_req, qx, n_qrm, enc_nq, own_agent)
 *   h, begin, wait, act_ptr, bufs_ptr, out_ptr: addresses (ints); names / agents / rms / getl: lists of A;
 *   labels: list of A lists (RM label by state index); action_index: dict name -> 0..4; qrm_req: the engine was
 *   built with the QRM columns; qx: their per-agent width (0: none); n_qrm / enc_nq: lists of A ints (the
 *   experiences per agent, the state encoder's stride); own_agent: rmx.compat.AgentRL, whose set_position and
 *   get_learning_algorithm this module performs itself for agents of exactly that class (the same attribute reads and
 *   writes, without an interpreter frame); agents of any other class get the method calls. */
/* dict(d): a copy of an exact dict (what dict(d) returns for one), the constructor for anything else */
static PyObject* dict_of(PyObject* d) {
  return PyDict_CheckExact(d) ? PyDict_Copy(d) : PyObject_CallOneArg((PyObject*)&PyDict_Type, d);
}

static long floordiv(long a, long b) { return a >= 0 ? a / b : -((-a + b - 1) / b); } /* Python's // for b > 0 */

/* infos["qrm_experience"] of agent i: one ten-field tuple per hypothetical RM state j < n_qrm[i]
 * (rm_environment_wrapper.py:168-179): (s, a, Renv + r, s', done, x·y cell, q, x'·y' cell, q', r) as rmx/compat.py's
 * _qrm_tuples builds them, from the QRM columns after the output record's head: s, s' [A][qx] i32, r [A][qx] f32,
 * done [A][qx] u8. */
static PyObject* qrm_tuples(const unsigned char* out, Py_ssize_t A, long qx, Py_ssize_t i, int32_t action, double renv,
                            PyObject* n_qrm, PyObject* enc_nq) {
  const long nj = PyLong_AsLong(PyList_GET_ITEM(n_qrm, i)), nq = PyLong_AsLong(PyList_GET_ITEM(enc_nq, i));
  if (PyErr_Occurred()) return NULL;
  if (nq <= 0 || nj < 0 || nj > qx) {
    PyErr_SetString(PyExc_ValueError, "dict_step: bad QRM layout");
    return NULL;
  }
  const size_t head = 4 * (6 * (size_t)A + 1), n = (size_t)A * (size_t)qx;
  PyObject* lst = PyList_New(nj);
  if (!lst) return NULL;
  for (long j = 0; j < nj; ++j) {
    const size_t o = (size_t)i * (size_t)qx + (size_t)j;
    int32_t s_, sn;
    float hr;
    memcpy(&s_, out + head + 4 * o, 4);
    memcpy(&sn, out + head + 4 * (n + o), 4);
    memcpy(&hr, out + head + 4 * (2 * n + o), 4);
    const int done = out[head + 12 * n + o] != 0;
    /* Python floor division / modulo of the encoded states (non-negative: a cell times the stride plus q) */
    const long fs = floordiv(s_, nq), fsn = floordiv(sn, nq);
    PyObject* t = Py_BuildValue("(iidiOlllld)", (int)s_, (int)action, renv + (double)hr, (int)sn,
                                done ? Py_True : Py_False, fs, (long)s_ - fs * nq, fsn, (long)sn - fsn * nq, (double)hr);
    if (!t) {
      Py_DECREF(lst);
      return NULL;
    }
    PyList_SET_ITEM(lst, j, t);
  }
  return lst;
}

static PyObject* dict_step(PyObject* self, PyObject* args) {
  PyObject *ctx, *actions;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!O", &PyTuple_Type, &ctx, &actions)) return NULL;
  if (PyTuple_GET_SIZE(ctx) != CTX_ITEMS) {
    PyErr_SetString(PyExc_ValueError, "dict_step: bad context");
    return NULL;
  }
  void* h = PyLong_AsVoidPtr(PyTuple_GET_ITEM(ctx, 0));
  begin_fn begin = (begin_fn)PyLong_AsVoidPtr(PyTuple_GET_ITEM(ctx, 1));
  wait_fn wait = (wait_fn)PyLong_AsVoidPtr(PyTuple_GET_ITEM(ctx, 2));
  int32_t* act = (int32_t*)PyLong_AsVoidPtr(PyTuple_GET_ITEM(ctx, 3));
  void* bufs = PyLong_AsVoidPtr(PyTuple_GET_ITEM(ctx, 4));
  const unsigned char* out = (const unsigned char*)PyLong_AsVoidPtr(PyTuple_GET_ITEM(ctx, 5));
  if (PyErr_Occurred()) return NULL;
  const int fl_kind = PyObject_IsTrue(PyTuple_GET_ITEM(ctx, 6));
  const int fl_slip = PyObject_IsTrue(PyTuple_GET_ITEM(ctx, 7));
  if (fl_kind < 0 || fl_slip < 0) return NULL;
  PyObject *names = PyTuple_GET_ITEM(ctx, 8), *agents = PyTuple_GET_ITEM(ctx, 9), *rms = PyTuple_GET_ITEM(ctx, 10);
  PyObject *labels = PyTuple_GET_ITEM(ctx, 11), *getl = PyTuple_GET_ITEM(ctx, 12), *env = PyTuple_GET_ITEM(ctx, 13);
  PyObject* action_index = PyTuple_GET_ITEM(ctx, 14);
  const int qrm_req = PyObject_IsTrue(PyTuple_GET_ITEM(ctx, 15));
  const long qx = PyLong_AsLong(PyTuple_GET_ITEM(ctx, 16));
  PyObject *n_qrm = PyTuple_GET_ITEM(ctx, 17), *enc_nq = PyTuple_GET_ITEM(ctx, 18);
  if (qrm_req < 0 || PyErr_Occurred()) return NULL;
  if (!PyList_Check(names) || !PyList_Check(agents) || !PyList_Check(rms) || !PyList_Check(labels) ||
      !PyList_Check(getl) || !PyDict_Check(action_index) || !PyList_Check(n_qrm) || !PyList_Check(enc_nq)) {
    PyErr_SetString(PyExc_TypeError, "dict_step: bad context types");
    return NULL;
  }
  if (!PyDict_Check(actions)) Py_RETURN_NONE; /* another mapping type: the Python path */
  const Py_ssize_t A = PyList_GET_SIZE(names);
  if (A < 1 || A > MAXA || PyList_GET_SIZE(agents) != A || PyList_GET_SIZE(rms) != A || PyList_GET_SIZE(labels) != A ||
      PyList_GET_SIZE(getl) != A || PyList_GET_SIZE(n_qrm) != A || PyList_GET_SIZE(enc_nq) != A) {
    PyErr_SetString(PyExc_ValueError, "dict_step: agent lists disagree");
    return NULL;
  }
  /* rm_environment_wrapper.py:78: getattr(agent.get_learning_algorithm(), "use_qrm", False), every step */
  /* (LOOKUP_ATTR: a missing attribute is no exception, as getattr(x, name, default) — no error object is built for
   * the common learner-less or use_qrm-less case) */
  PyObject* own_agent = PyTuple_GET_ITEM(ctx, 19);
  int use_qrm[MAXA] = {0};
  for (Py_ssize_t i = 0; i < A; ++i) {
    PyObject* g = PyList_GET_ITEM(getl, i);
    PyObject* learner = NULL;
    /* AgentRL.get_learning_algorithm is getattr(self, "learning_algorithm", None) */
    if (g == Py_None || (PyObject*)Py_TYPE(PyList_GET_ITEM(agents, i)) == own_agent) {
      if (LOOKUP_ATTR(PyList_GET_ITEM(agents, i), s_learning_algorithm, &learner) < 0) return NULL;
      if (!learner) continue;
    } else if (!(learner = PyObject_CallNoArgs(g))) {
      return NULL;
    }
    PyObject* u = NULL;
    const int found = LOOKUP_ATTR(learner, s_use_qrm, &u);
    Py_DECREF(learner);
    if (found < 0) return NULL;
    if (!u) continue;
    const int t = PyObject_IsTrue(u);
    Py_DECREF(u);
    if (t < 0) return NULL;
    if (t && !qrm_req) Py_RETURN_NONE; /* QRM turned on since the build: the Python path rebuilds the engine */
    use_qrm[i] = t;
  }
  /* the actions: actions[agent.name].name -> index (anything else: the Python path, which raises as it does) */
  int32_t k[MAXA];
  for (Py_ssize_t i = 0; i < A; ++i) {
    PyObject* a = PyDict_GetItemWithError(actions, PyList_GET_ITEM(names, i));
    if (!a) {
      if (PyErr_Occurred()) return NULL;
      Py_RETURN_NONE;
    }
    Py_INCREF(a); /* borrowed from the caller's dict: held while .name (a property, maybe) runs */
    PyObject* nm = PyObject_GetAttr(a, s_name);
    Py_DECREF(a);
    if (!nm) {
      PyErr_Clear();
      Py_RETURN_NONE;
    }
    PyObject* ix = PyDict_GetItemWithError(action_index, nm);
    Py_DECREF(nm);
    if (!ix) {
      if (PyErr_Occurred()) PyErr_Clear();
      Py_RETURN_NONE;
    }
    const long kv = PyLong_AsLong(ix);
    if (kv == -1 && PyErr_Occurred()) return NULL;
    if (kv < 0 || kv > 4) Py_RETURN_NONE; /* not an action index: the Python path (its ValueError) */
    k[i] = (int32_t)kv;
    if (k[i] == 4 && fl_slip) Py_RETURN_NONE; /* the reference's KeyError path */
  }
  for (Py_ssize_t i = 0; i < A; ++i) act[i] = k[i];
  /* the request goes out; the bookkeeping of the previous state overlaps its round trip */
  int rc = begin(h, act, 0, NULL);
  if (rc) return PyLong_FromLong(rc);
  PyObject *prev[MAXA] = {0}, *prev_q[MAXA] = {0}, *full[MAXA] = {0};
  PyObject *active = NULL, *fail = NULL, *steps = NULL, *res = NULL;
  PyObject *obs = NULL, *rewards = NULL, *terms = NULL, *truncs = NULL, *infos = NULL;
  active = PyObject_GetAttr(env, s_active_agents);
  fail = active ? PyObject_GetAttr(env, s_agent_fail) : NULL;
  steps = fail ? PyObject_GetAttr(env, s_agent_steps) : NULL;
  int ok = steps != NULL;
  for (Py_ssize_t i = 0; ok && i < A; ++i) {
    PyObject* st = PyObject_GetAttr(PyList_GET_ITEM(agents, i), s_state);
    prev[i] = st ? dict_of(st) : NULL; /* dict(ag.state) */
    Py_XDECREF(st);
    prev_q[i] = prev[i] ? PyObject_GetAttr(PyList_GET_ITEM(rms, i), s_current_state) : NULL;
    ok = prev_q[i] != NULL;
    if (ok && !fl_kind) { /* OW skips inactive agents before filling infos (ma_office.py:143-144) */
      PyObject* v = PyObject_CallMethod(active, "get", "OO", PyList_GET_ITEM(names, i), Py_True);
      ok = v != NULL;
      full[i] = v;
    }
  }
  obs = PyDict_New();
  rewards = PyDict_New();
  terms = PyDict_New();
  truncs = PyDict_New();
  infos = PyDict_New();
  ok = ok && obs && rewards && terms && truncs && infos;
  /* wait even when the bookkeeping failed: the request is outstanding.  The interpreter lock is released for the
   * round trip, as a ctypes call releases it (the Python path). */
  Py_BEGIN_ALLOW_THREADS
  rc = wait(h, bufs);
  Py_END_ALLOW_THREADS
  if (rc) {
    if (ok) res = PyLong_FromLong(rc);
    goto done;
  }
  if (!ok) goto done;
  {
    /* the record: x [A], y [A], q [A], flags [A] i32, reward [A], renv [A] f32, t i32 (rmx/compat.py _io_setup) */
    int32_t iv[4 * MAXA];
    float fv[2 * MAXA];
    int32_t t;
    memcpy(iv, out, sizeof(int32_t) * 4 * (size_t)A);
    memcpy(fv, out + 16 * A, sizeof(float) * 2 * (size_t)A);
    memcpy(&t, out + 24 * A, sizeof(int32_t));
    for (Py_ssize_t i = 0; i < A; ++i) {
      PyObject *name = PyList_GET_ITEM(names, i), *ag = PyList_GET_ITEM(agents, i), *rm = PyList_GET_ITEM(rms, i);
      const int32_t x = iv[i], y = iv[A + i], qi = iv[2 * A + i];
      const uint32_t f = (uint32_t)iv[3 * A + i];
      const double reward = (double)fv[i], renv = (double)fv[A + i];
      PyObject* lab = PyList_GET_ITEM(labels, i);
      if (qi < 0 || qi >= PyList_GET_SIZE(lab)) {
        PyErr_SetString(PyExc_RuntimeError, "dict_step: RM state index out of range");
        goto done;
      }
      PyObject* q = PyList_GET_ITEM(lab, qi);
      PyObject *px = PyLong_FromLong(x), *py = PyLong_FromLong(y);
      int pe;
      if ((PyObject*)Py_TYPE(ag) == own_agent) { /* AgentRL.set_position: position = (x, y); state = {pos_x, pos_y} */
        PyObject* pos = px && py ? PyTuple_Pack(2, px, py) : NULL;
        PyObject* sd = pos ? PyDict_New() : NULL;
        pe = !sd || PyDict_SetItem(sd, k_pos_x, px) || PyDict_SetItem(sd, k_pos_y, py) ||
             PyObject_SetAttr(ag, s_position, pos) || PyObject_SetAttr(ag, s_state, sd);
        Py_XDECREF(pos);
        Py_XDECREF(sd);
      } else {
        PyObject* r = px && py ? PyObject_CallMethodObjArgs(ag, s_set_position, px, py, NULL) : NULL;
        pe = !r;
        Py_XDECREF(r);
      }
      Py_XDECREF(px);
      Py_XDECREF(py);
      if (pe) goto done;
      if (PyObject_SetAttr(rm, s_current_state, q) < 0) goto done;
      PyObject* state = PyObject_GetAttr(ag, s_state);
      if (!state) goto done;
      int e = PyDict_SetItem(obs, name, state);
      PyObject* rw = PyFloat_FromDouble(reward);
      e = e || !rw || PyDict_SetItem(rewards, name, rw);
      Py_XDECREF(rw);
      e = e || PyDict_SetItem(terms, name, (f & 4u) ? Py_True : Py_False);  /* RMX_F_TERM */
      e = e || PyDict_SetItem(truncs, name, (f & 8u) ? Py_True : Py_False); /* RMX_F_TRUNC */
      PyObject* info = e ? NULL : PyDict_New();
      PyObject *rq = PyFloat_FromDouble(reward - renv), *re = NULL, *sc = NULL;
      e = e || !info || !rq;
      const int full_t = (!fl_kind && full[i]) ? PyObject_IsTrue(full[i]) : 0;
      e = e || full_t < 0; /* (a failing __bool__: its exception is returned) */
      const int fill = fl_kind || full_t == 1;
      if (!e && fill) {
        sc = dict_of(state); /* dict(state) */
        re = PyFloat_FromDouble(renv);
        e = !sc || !re || PyDict_SetItem(info, k_prev_s, prev[i]) || PyDict_SetItem(info, k_s, sc) ||
            PyDict_SetItem(info, k_Renv, re);
      }
      e = e || PyDict_SetItem(info, k_RQ, rq) || PyDict_SetItem(info, k_prev_q, prev_q[i]) ||
          PyDict_SetItem(info, k_q, q) || PyDict_SetItem(info, k_reward_machine, rm);
      if (!e && use_qrm[i] && qx > 0) { /* rm_environment_wrapper.py:78-89, the tuples of :168-179 */
        PyObject* ex = qrm_tuples(out, A, qx, i, k[i], renv, n_qrm, enc_nq);
        e = !ex || PyDict_SetItem(info, k_qrm_experience, ex);
        Py_XDECREF(ex);
      }
      e = e || PyDict_SetItem(info, k_env_terminated, (f & 16u) ? Py_True : Py_False) || /* RMX_F_ENV_TERM */
          PyDict_SetItem(info, k_rm_terminated, (f & 32u) ? Py_True : Py_False) ||  /* RMX_F_RM_TERM */
          PyDict_SetItem(infos, name, info);
      Py_XDECREF(sc);
      Py_XDECREF(re);
      Py_XDECREF(rq);
      Py_XDECREF(info);
      Py_DECREF(state);
      if (e) goto done;
      PyObject* st = PyLong_FromUnsignedLong(f >> 16); /* RMX_F_STEPS_SHIFT */
      e = !st || PyObject_SetItem(active, name, (f & 1u) ? Py_True : Py_False) ||
          PyObject_SetItem(fail, name, (f & 2u) ? Py_True : Py_False) || PyObject_SetItem(steps, name, st);
      Py_XDECREF(st);
      if (e) goto done;
    }
    PyObject* tv = PyLong_FromLong(t);
    if (!tv || PyObject_SetAttr(env, s_timestep, tv) < 0) {
      Py_XDECREF(tv);
      goto done;
    }
    Py_DECREF(tv);
    res = PyTuple_Pack(5, obs, rewards, terms, truncs, infos);
  }
done:
  for (Py_ssize_t i = 0; i < A; ++i) {
    Py_XDECREF(prev[i]);
    Py_XDECREF(prev_q[i]);
    Py_XDECREF(full[i]);
  }
  Py_XDECREF(active);
  Py_XDECREF(fail);
  Py_XDECREF(steps);
  Py_XDECREF(obs);
  Py_XDECREF(rewards);
  Py_XDECREF(terms);
  Py_XDECREF(truncs);
  Py_XDECREF(infos);
  return res;
}

static PyMethodDef methods[] = {
    {"step", dict_step, METH_VARARGS, "step(ctx, actions): the dict-API step of rmx.compat (see the module source)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_dictstep", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__dictstep(void) {
#define INTERN(v, s) \
  if (!(v = PyUnicode_InternFromString(s))) return NULL
  INTERN(s_name, "name");
  INTERN(s_use_qrm, "use_qrm");
  INTERN(s_state, "state");
  INTERN(s_current_state, "current_state");
  INTERN(s_set_position, "set_position");
  INTERN(s_active_agents, "active_agents");
  INTERN(s_agent_fail, "agent_fail");
  INTERN(s_agent_steps, "agent_steps");
  INTERN(s_timestep, "timestep");
  INTERN(s_learning_algorithm, "learning_algorithm");
  INTERN(s_position, "position");
  INTERN(k_pos_x, "pos_x");
  INTERN(k_pos_y, "pos_y");
  INTERN(k_prev_s, "prev_s");
  INTERN(k_s, "s");
  INTERN(k_Renv, "Renv");
  INTERN(k_RQ, "RQ");
  INTERN(k_prev_q, "prev_q");
  INTERN(k_q, "q");
  INTERN(k_reward_machine, "reward_machine");
  INTERN(k_env_terminated, "env_terminated");
  INTERN(k_rm_terminated, "rm_terminated");
  INTERN(k_qrm_experience, "qrm_experience");
#undef INTERN
  PyObject* m = PyModule_Create(&module);
  if (!m) return NULL;
  /* what rmx/compat.py checks before it uses the module: the context layout and the source it was built from */
  if (PyModule_AddIntConstant(m, "CTX_ITEMS", CTX_ITEMS) < 0 ||
      PyModule_AddStringConstant(m, "SOURCE_HASH", RMX_DICTSTEP_HASH) < 0) {
    Py_DECREF(m);
    return NULL;
  }
  return m;
}
