#include "api/storage.h"

#include <openssl/sha.h>

#include <algorithm>
#include <cstdio>

#include "common/quantity.h"

namespace xsched {

namespace {

int64_t storage_bytes(const Json& v) {
  if (v.is_string()) {
    Quantity q;
    if (Quantity::try_parse(v.as_string(), &q)) return q.value();
    return 0;
  }
  return v.as_int(0);
}

std::vector<std::string> strings(const Json& a) {
  std::vector<std::string> out;
  for (const auto& s : a.items()) out.push_back(s.as_string());
  return out;
}

SelOp sel_op(const std::string& s) {
  if (s == "NotIn") return SelOp::NotIn;
  if (s == "Exists") return SelOp::Exists;
  if (s == "DoesNotExist") return SelOp::DoesNotExist;
  if (s == "Gt") return SelOp::Gt;
  if (s == "Lt") return SelOp::Lt;
  return SelOp::In;
}

NodeSelectorTerm parse_node_term(const Json& t) {
  NodeSelectorTerm term;
  for (const auto* key : {"matchExpressions", "matchFields"}) {
    auto& dst = std::string(key) == "matchExpressions" ? term.match_expressions : term.match_fields;
    for (const auto& r : t[key].items()) {
      SelectorRequirement req;
      req.key = r["key"].as_string();
      req.op = sel_op(r["operator"].as_string());
      req.values = strings(r["values"]);
      dst.push_back(std::move(req));
    }
  }
  return term;
}

// The in-tree source of a PV spec or a pod volume, if it is one we track.
InTree intree_source(const Json& src, std::string* id, bool* ro, std::vector<std::string>* mons, std::string* pool) {
  if (const Json* v = src.get("awsElasticBlockStore")) {
    *id = (*v)["volumeID"].as_string();
    *ro = (*v)["readOnly"].as_bool(false);
    return InTree::AWSEBS;
  }
  if (const Json* v = src.get("gcePersistentDisk")) {
    *id = (*v)["pdName"].as_string();
    *ro = (*v)["readOnly"].as_bool(false);
    return InTree::GCEPD;
  }
  if (const Json* v = src.get("azureDisk")) {
    *id = (*v)["diskName"].as_string();
    *ro = (*v)["readOnly"].as_bool(false);
    return InTree::AzureDisk;
  }
  if (const Json* v = src.get("cinder")) {
    *id = (*v)["volumeID"].as_string();
    *ro = (*v)["readOnly"].as_bool(false);
    return InTree::Cinder;
  }
  if (const Json* v = src.get("iscsi")) {
    *id = (*v)["iqn"].as_string();
    *ro = (*v)["readOnly"].as_bool(false);
    return InTree::ISCSI;
  }
  if (const Json* v = src.get("rbd")) {
    *id = (*v)["image"].as_string();
    *ro = (*v)["readOnly"].as_bool(false);
    if (mons) *mons = strings((*v)["monitors"]);
    if (pool) *pool = (*v)["pool"].str_or("rbd");
    return InTree::RBD;
  }
  return InTree::None;
}

}  // namespace

const char* intree_plugin_name(InTree k) {
  switch (k) {
    case InTree::AWSEBS: return "kubernetes.io/aws-ebs";
    case InTree::GCEPD: return "kubernetes.io/gce-pd";
    case InTree::AzureDisk: return "kubernetes.io/azure-disk";
    case InTree::Cinder: return "kubernetes.io/cinder";
    case InTree::ISCSI: return "kubernetes.io/iscsi";
    case InTree::RBD: return "kubernetes.io/rbd";
    default: return "";
  }
}

std::vector<PodVolume> parse_pod_volumes(const Json& spec, const std::string& pod_name) {
  std::vector<PodVolume> out;
  for (const auto& v : spec["volumes"].items()) {
    PodVolume pv;
    pv.name = v["name"].as_string();
    if (const Json* c = v.get("persistentVolumeClaim")) {
      pv.kind = PodVolume::Kind::PVC;
      pv.claim = (*c)["claimName"].as_string();
      pv.read_only = (*c)["readOnly"].as_bool(false);
    } else if (v.get("ephemeral")) {
      // Generic ephemeral volume: its PVC is "<pod name>-<volume name>"
      // (component-helpers/storage/ephemeral.VolumeClaimName).
      pv.kind = PodVolume::Kind::Ephemeral;
      pv.claim = pod_name + "-" + pv.name;
    } else {
      pv.intree = intree_source(v, &pv.id, &pv.read_only, &pv.rbd_monitors, &pv.rbd_pool);
      if (pv.intree == InTree::None) continue;  // emptyDir, configMap, hostPath, ...: nothing to schedule on
      pv.kind = PodVolume::Kind::InTree;
    }
    out.push_back(std::move(pv));
  }
  return out;
}

// ------------------------------------------------------------------- PV ---
bool PersistentVolume::matches_node(const Node& n) const {
  if (!has_node_affinity) return true;
  for (const auto& t : node_affinity)
    if (node_selector_term_matches(t, n)) return true;
  return false;
}

std::shared_ptr<PersistentVolume> PersistentVolume::from_json(const Json& obj) {
  auto pv = std::make_shared<PersistentVolume>();
  pv->meta = ObjectMeta::from_json(obj);
  const Json& spec = obj["spec"];
  if (spec["storageClassName"].is_string())
    pv->storage_class = spec["storageClassName"].as_string();
  else if (const std::string* a = pv->meta.annotation(kAnnStorageClassBeta))
    pv->storage_class = *a;
  pv->capacity = storage_bytes(spec["capacity"]["storage"]);
  pv->access_modes = strings(spec["accessModes"]);
  if (spec["volumeMode"].is_string()) pv->volume_mode = spec["volumeMode"].as_string();
  pv->phase = obj["status"]["phase"].as_string();
  if (const Json* cr = spec.get("claimRef"); cr && cr->is_object()) {
    pv->has_claim_ref = true;
    pv->claim_ns = (*cr)["namespace"].as_string();
    pv->claim_name = (*cr)["name"].as_string();
    pv->claim_uid = (*cr)["uid"].as_string();
  }
  if (const Json* req = spec.path({"nodeAffinity", "required"})) {
    pv->has_node_affinity = true;
    for (const auto& t : (*req)["nodeSelectorTerms"].items()) pv->node_affinity.push_back(parse_node_term(t));
  }
  if (const Json* csi = spec.get("csi")) {
    pv->csi_driver = (*csi)["driver"].as_string();
    pv->csi_handle = (*csi)["volumeHandle"].as_string();
  } else {
    bool ro = false;
    pv->intree = intree_source(spec, &pv->intree_id, &ro, nullptr, nullptr);
  }
  return pv;
}

// ------------------------------------------------------------------ PVC ---
std::shared_ptr<PersistentVolumeClaim> PersistentVolumeClaim::from_json(const Json& obj) {
  auto c = std::make_shared<PersistentVolumeClaim>();
  c->meta = ObjectMeta::from_json(obj);
  const Json& spec = obj["spec"];
  // storagehelpers.GetPersistentVolumeClaimClass: the beta annotation wins.
  if (const std::string* a = c->meta.annotation(kAnnStorageClassBeta)) {
    c->has_class = true;
    c->storage_class = *a;
  } else if (spec["storageClassName"].is_string()) {
    c->has_class = true;
    c->storage_class = spec["storageClassName"].as_string();
  }
  c->volume_name = spec["volumeName"].as_string();
  c->request = storage_bytes(spec["resources"]["requests"]["storage"]);
  c->access_modes = strings(spec["accessModes"]);
  if (spec["volumeMode"].is_string()) c->volume_mode = spec["volumeMode"].as_string();
  c->selector = LabelSelector::from_json(spec.get("selector"));
  c->phase = obj["status"]["phase"].as_string();
  for (const auto& o : obj["metadata"]["ownerReferences"].items())
    if (o["controller"].as_bool(false)) {
      c->controller_uid = o["uid"].as_string();
      c->controller_kind = o["kind"].as_string();
    }
  return c;
}

// --------------------------------------------------------- StorageClass ---
bool StorageClass::topology_matches(const Node& n) const {
  if (allowed_topologies.empty()) return true;
  for (const auto& t : allowed_topologies) {
    bool all = true;
    for (const auto& [key, values] : t.exprs) {
      const std::string* v = n.meta.label(key);
      if (!v || std::find(values.begin(), values.end(), *v) == values.end()) {
        all = false;
        break;
      }
    }
    if (all) return true;
  }
  return false;
}

std::shared_ptr<StorageClass> StorageClass::from_json(const Json& obj) {
  auto sc = std::make_shared<StorageClass>();
  sc->meta = ObjectMeta::from_json(obj);
  sc->provisioner = obj["provisioner"].as_string();
  if (obj["volumeBindingMode"].is_string()) {
    sc->binding_mode_set = true;
    sc->wait_for_first_consumer = obj["volumeBindingMode"].as_string() == "WaitForFirstConsumer";
  }
  for (const auto& t : obj["allowedTopologies"].items()) {
    TopologySelectorTerm term;
    for (const auto& e : t["matchLabelExpressions"].items()) term.exprs.emplace_back(e["key"].as_string(), strings(e["values"]));
    sc->allowed_topologies.push_back(std::move(term));
  }
  return sc;
}

// -------------------------------------------------------------- CSINode ---
bool CSINode::migrated(InTree k) const {
  const std::string* a = meta.annotation(kAnnMigratedPlugins);
  if (!a || k == InTree::None) return false;
  const std::string want = intree_plugin_name(k);
  size_t start = 0;
  while (start <= a->size()) {
    size_t end = a->find(',', start);
    if (end == std::string::npos) end = a->size();
    if (a->compare(start, end - start, want) == 0) return true;
    start = end + 1;
  }
  return false;
}

std::shared_ptr<CSINode> CSINode::from_json(const Json& obj) {
  auto n = std::make_shared<CSINode>();
  n->meta = ObjectMeta::from_json(obj);
  for (const auto& d : obj["spec"]["drivers"].items()) {
    Driver dr;
    dr.name = d["name"].as_string();
    if (const Json* c = d.path({"allocatable", "count"}); c && c->is_number()) {
      dr.has_count = true;
      dr.count = c->as_int();
    }
    n->drivers.push_back(std::move(dr));
  }
  return n;
}

std::string csi_attach_limit_key(const std::string& driver) {
  static const std::string kPrefix = "attachable-volumes-csi-";
  constexpr size_t kResourceNameLengthLimit = 63;
  if (kPrefix.size() + driver.size() < kResourceNameLengthLimit) return kPrefix + driver;
  unsigned char md[SHA_DIGEST_LENGTH];
  SHA1(reinterpret_cast<const unsigned char*>(driver.data()), driver.size(), md);
  char hex[2 * SHA_DIGEST_LENGTH + 1];
  for (int i = 0; i < SHA_DIGEST_LENGTH; ++i) std::snprintf(hex + 2 * i, 3, "%02x", md[i]);
  return kPrefix + driver.substr(0, 23) + std::string(hex, 16);
}

}  // namespace xsched
